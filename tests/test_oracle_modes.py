"""CPU checks of the oracle's restatement of the opt-in GL-path modes (orc_render_p_ex):
properties that pin it to the plain Mode P oracle (itself pinned to the reference's
goldens) where the modes must not matter, and the GL path's defining behaviour where
they must. The GL path cannot run here, so the modes are "parity unpinned" beyond these
properties."""
import numpy as np

import oracle


def _scene_without_lights():
    s, m = oracle.default_scene_arrays()
    m = np.array(m, np.float32).reshape(-1, 9)
    m[:, 4:7] = 0.0   # no emissive anywhere
    return s, m.ravel()


def test_no_double_light_is_identity_without_emitters():
    s, m = _scene_without_lights()
    a, ra = oracle.orc_render(96, 54, frames=3, depth=8, spheres=s, mats=m)
    b, rb = oracle.orc_render_ex(96, 54, frames=3, depth=8, spheres=s, mats=m, flags=64)
    assert ra == rb and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_no_double_light_removes_light_only():
    a, ra = oracle.orc_render(96, 54, frames=3, depth=8)
    b, rb = oracle.orc_render_ex(96, 54, frames=3, depth=8, flags=64)
    assert ra == rb                       # same paths, same rays: only emission changes
    assert not np.array_equal(a, b)
    assert (b[..., :3] <= a[..., :3] + 1e-5).mean() > 0.999   # emission removed, not added


def test_features_do_not_change_colour_and_start_at_zero_spread():
    feats = {n: np.zeros((54, 96, 4), np.float32) for n in oracle.FEATURE_NAMES}
    a, ra = oracle.orc_render(96, 54, frames=1, depth=8)
    b, rb = oracle.orc_render_ex(96, 54, frames=1, depth=8, features=feats)
    assert ra == rb and np.array_equal(a.view(np.uint32), b.view(np.uint32))
    for n in ("color_std", "normal_std", "world_pos_std"):
        assert not feats[n].any(), n      # frame 0: mean == sample, so the spread is 0
    nrm = feats["normal"][..., :3]
    hit = np.abs(nrm).sum(-1) > 0
    assert hit.mean() > 0.5
    assert np.allclose(np.linalg.norm(nrm[hit], axis=-1), 1.0, atol=1e-5)   # unit first-hit normals


def test_features_stop_after_max_frame():
    feats = {n: np.zeros((36, 64, 4), np.float32) for n in oracle.FEATURE_NAMES}
    oracle.orc_render_ex(64, 36, frames=3, depth=8, features=feats, max_frame=2)
    snap = {n: b.copy() for n, b in feats.items()}
    buf = np.zeros((36, 64, 4), np.float32)
    oracle.orc_render_ex(64, 36, frames=2, frame0=3, depth=8, buf=buf, features=feats, max_frame=2)
    for n in oracle.FEATURE_NAMES:
        assert np.array_equal(feats[n], snap[n]), n


def test_misses_give_zero_features():
    s = np.array([0.0, -1000.0, 0.0, 0.5], np.float32)        # one sphere far out of view
    m = np.array([0, 0.5, 0.5, 0.5, 0, 0, 0, 0, 0], np.float32)
    feats = {n: np.full((18, 32, 4), 7.0, np.float32) for n in ("normal", "world_pos", "albedo")}
    oracle.orc_render_ex(32, 18, frames=1, depth=8, spheres=s, mats=m, features=feats)
    for n, b in feats.items():
        assert not b[..., :3].any(), n   # frame 0 lerp: 7*0 + 0*1
        assert (b[..., 3] == 7.0).all()
