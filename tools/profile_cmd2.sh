#!/bin/bash
# rocprofv3 evidence for an arbitrary command, each pass its own run: kernel trace + stats, then PMC
# passes — instruction mix, issue / wait cycles, VALU flops, LDS bank conflicts and waits, the
# instruction cache (the interpreter's code size against the per-CU-pair I-cache), HBM bytes.
#   tools/profile_cmd2.sh OUTDIR python3 tools/microbench.py C2-complete
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$1; shift
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- "$@" > $OUT/kt.log 2>&1 || exit $?
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES" \
           "SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FMA_F32 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_MUL_F64" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_IFETCH SQ_INST_CYCLES_SALU" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o pmc$i -- "$@" > $OUT/pmc$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then  # (a failed pass ends the script: nothing more runs on the GPU after it)
    echo "pmc pass $i ($pmc) failed: $rc" >> $OUT/errors.txt
    python3 tools/pmc_summary.py $OUT > $OUT/summary.txt
    exit $rc
  fi
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt
exit 0
