"""bench.py's workload definition (CPU): strong scaling keeps BASELINE's frame fixed at
every N (config 2 stays 1280x720 at 4 spp, config 5 renders 256 spp in total), weak
scaling multiplies the samples by N; and the roofline inputs the committed profiles give."""
import json
import os

import pytest

import bench


@pytest.mark.parametrize("config,spp", [(2, 4), (3, 16), (4, 64), (5, 256)])
@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_strong_scaling_keeps_the_frame(config, spp, n):
    w = bench.workload(config, n, "strong")
    assert w["spp_total"] == spp and w["shards"] == n
    assert w["pixel_samples_total"] == w["width"] * w["height"] * spp


@pytest.mark.parametrize("n", [1, 2, 8])
def test_weak_scaling_multiplies_samples(n):
    w = bench.workload(2, n, "weak")
    assert w["spp_total"] == 4 * n


def test_default_is_strong_and_config2():
    import argparse  # noqa: F401  (parse the real parser's defaults)
    src = open(bench.__file__).read()
    assert 'choices=["strong", "weak"], default="strong"' in src
    assert "--config\", type=int, default=2" in src


def test_diagnostic_overrides():
    w = bench.workload(4, 1, "strong", spp=2, depth=3, shard_of=8)
    assert (w["spp_total"], w["depth"], w["shards"]) == (2, 3, 8)


def test_committed_pmc_summaries_are_consistent():
    """Every profile bench.py may read carries the fields its roofline uses, and its
    lane-op count is SQ_INSTS_VALU x 64 x lane_util."""
    idx_path = bench.PMC_INDEX
    if not os.path.exists(idx_path):
        pytest.skip("no committed PMC index yet")
    idx = json.load(open(idx_path))
    assert idx
    for key in idx:
        s = bench.read_pmc(key)
        assert s is not None, key
        c = s["counters_per_launch"]
        lu = c["SQ_THREAD_CYCLES_VALU"] / (c["SQ_ACTIVE_INST_VALU"] * 64)
        assert abs(s["lane_util"] - lu) < 1e-3
        assert abs(s["lane_ops_per_launch"] - c["SQ_INSTS_VALU"] * 64 * lu) <= 1e-6 * s["lane_ops_per_launch"]
        assert s["hbm_bytes_per_launch"] == 2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024
        assert s["kernel_trace"]["avg_ns"] > 0


def test_default_steps_give_a_long_timed_region():
    """Without --steps the timed region is tens of ms at every config (config 2: 200 steps of
    ~0.22 ms; 20 steps measured the launch and drain edges at ~8 % of the region)."""
    assert bench.DEFAULT_STEPS[2] == 200
    approx_ms = {2: 0.22, 3: 1.8, 4: 84.0, 5: 1370.0}
    for c, ms in approx_ms.items():
        assert bench.DEFAULT_STEPS[c] * ms >= 40.0, c
