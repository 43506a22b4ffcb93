# SQ counters for two builds of the plan selected by an env switch: A = default, B = $ABVAR=0
# usage: ABVAR=DNN_HIP_CONV0_PACKED bash tools/sq_ab_job.sh   -> gpurun_out/sq_{a,b}_{def,off}
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp
B="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --precision ${PREC:-fp32}"
for tag in def off; do
  if [ $tag = off ]; then export $ABVAR=0; fi
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/sq_a_$tag -o a --output-format csv -- $B > $R/gpurun_out/sq_a_$tag.log 2>&1 || exit 1
  timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA -d $R/gpurun_out/sq_b_$tag -o b --output-format csv -- $B > $R/gpurun_out/sq_b_$tag.log 2>&1 || exit 1
done
echo SQOK
