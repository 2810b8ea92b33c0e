#!/bin/bash
# What the driver runs at round end: GPU test suite, smoke(), default bench.
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/roundend; mkdir -p $out
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-2} $out/$name.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pytest_gpu 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 run bench 300 python bench.py
