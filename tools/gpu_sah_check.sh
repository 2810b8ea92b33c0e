set -o pipefail
mkdir -p gpurun_out/sah
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_features.py -k "bvh or scene1000 or c4 or c5 or fuzz" > gpurun_out/sah/tests.log 2>&1 || { tail -30 gpurun_out/sah/tests.log; exit 1; }
tail -1 gpurun_out/sah/tests.log
CFGS="sah:6" tools/gpu_sah.sh
timeout -k 10 200 python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/sah/c3.log 2>&1 && grep '^{' gpurun_out/sah/c3.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('c3', d['value'], d['ms_per_step'])"
