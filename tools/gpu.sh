#!/bin/bash
# One parameterised GPU session (replaces round 1's one-off gpu_*.sh scripts).
#
#   TAG=r2_x gpurun -- bash tools/gpu.sh STEP [STEP ...]
#
# Steps (each under its own timeout; the session stops at the first failure):
#   test[=K]          pytest -m gpu (optionally -k K)
#   smoke             __graft_entry__.smoke()
#   bench=C[,ARGS]    bench.py --config C (ARGS: extra bench flags, ';'-separated)
#   trace=C[,ARGS]    rocprofv3 --kernel-trace --stats of bench.py --config C --streams 1
#   pmc=C,GROUP[,ARGS] one rocprofv3 --pmc pass (GROUP: fetch | write | sq | sq2 | cache) of bench --config C
#   py=SCRIPT[,ARGS]  python SCRIPT ARGS (diagnostics under tools/; NAME=VALUE tokens set the environment)
#   ab=V,C[,ARGS]     bench.py --config C with LRT_LIB=build_exp/liblrt_V.so (tools/build_variant.sh),
#                     timed region only (A/B of library variants; V=default: the in-tree library;
#                     NAME=VALUE tokens in ARGS set environment variables)
# Output: gpurun_out/$TAG/<step>.log (+ rocprof CSVs). BSTEPS: timed steps (default: bench.py's per-config default).
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-latest}
out=gpurun_out/$TAG
mkdir -p "$out"
export TMPDIR=/tmp
BSTEPS=${BSTEPS:-default}
STEPARG=(--steps "$BSTEPS")
[ "$BSTEPS" = default ] && STEPARG=()   # bench.py's per-config default
declare -A PMC=(
  [fetch]="FETCH_SIZE"
  [write]="WRITE_SIZE"
  [sq]="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY"
  [sq2]="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"
  [cache]="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"
)
run() {   # run NAME SECONDS CMD...
  local name=$1 t=$2
  shift 2
  local t0=$SECONDS
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($((SECONDS - t0)) s)"
  tail -n "${TAILN:-3}" "$out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
i=0
for s in "$@"; do
  i=$((i + 1))
  key=${s%%=*}
  val=${s#*=}
  [ "$val" = "$s" ] && val=""
  c=${val%%,*}
  rest=""
  [[ "$val" == *,* ]] && rest=${val#*,}
  extra=${rest//;/ }
  case $key in
    test)
      if [ -n "$val" ]; then
        run "test$i" 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "$val"
      else
        run "test$i" 1100 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
      fi ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) TAILN=1 run "bench_c${c}_$i" 600 python bench.py --config "$c" "${STEPARG[@]}" $extra ;;
    trace) run "trace_c${c}_$i" 600 rocprofv3 --kernel-trace --stats -d "$out" -o "trace_c${c}" --output-format csv -- \
             python3 bench.py --config "$c" "${STEPARG[@]}" --streams 1 --no-cpu-baseline $extra ;;
    pmc)   g=${rest%%,*}
           pextra=""
           [[ "$rest" == *,* ]] && pextra=${rest#*,}
           run "pmc_c${c}_$g" 300 rocprofv3 --pmc ${PMC[$g]} -d "$out" -o "pmc_c${c}_$g" --output-format csv -- \
             python3 bench.py --config "$c" --steps 2 --warmup 2 --streams 1 --no-cpu-baseline --no-extra-legs ${pextra//;/ } ;;
    py)    penv=() pargs=()   # NAME=VALUE tokens are environment settings (e.g. LRT_LIB=...)
           for tok in ${val//,/ }; do
             if [[ "$tok" =~ ^[A-Z_][A-Z0-9_]*= ]]; then penv+=("$tok"); else pargs+=("$tok"); fi
           done
           run "py$i" 600 env "${penv[@]}" python "${pargs[@]}" ;;
    ab)    c2=${rest%%,*}
           extra2=""
           [[ "$rest" == *,* ]] && extra2=${rest#*,}
           lib=build_exp/liblrt_$c.so
           [ "$c" = default ] && lib=learnraytracing_amd/liblrt_hip.so
           envs=() bargs=()   # ARGS tokens NAME=VALUE are environment settings (e.g. LRT_BVH_LEAF=8)
           for tok in ${extra2//;/ }; do
             if [[ "$tok" =~ ^[A-Z_][A-Z0-9_]*= ]]; then envs+=("$tok"); else bargs+=("$tok"); fi
           done
           TAILN=1 run "ab_${c}_c${c2}_$i" 600 env LRT_LIB="$lib" "${envs[@]}" python bench.py --config "$c2" \
             "${STEPARG[@]}" --no-cpu-baseline --no-extra-legs "${bargs[@]}" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
