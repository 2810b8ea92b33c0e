#!/bin/bash
# Extended SQ/SQC counters for the given kernels (KERNELS="v0 v1"), one --pmc pass per group.
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/cnt; mkdir -p $out
export TMPDIR=/tmp
G1="SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"
G2="SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_LDS_BANK_CONFLICT"
G3="SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"
G4="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
for k in ${KERNELS:-v0 v1}; do
  i=0
  for g in "$G1" "$G2" "$G3" "$G4"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $g -d $out -o ${k}_g$i --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --kernel $k $BENCH_ARGS > $out/${k}_g$i.log 2>&1
    rc=$?; echo "$k g$i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $out/${k}_g$i.log; exit $rc; fi
  done
done
python3 tools/counter_table.py $out
