# SQ counters of the fp32 plan (x3 conv6/conv7): MFMA busy, waits, LDS conflicts, clock
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/x3sq; mkdir -p $O; cd /tmp
F="--steps 3 --warmup 1 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e"
B="python3 $R/bench.py $F"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/a -o a --output-format csv -- $B > $O/a.log 2>&1 || { tail -5 $O/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/b -o b --output-format csv -- $B > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/t -o t --output-format csv -- $B > $O/t.log 2>&1 || { tail -5 $O/t.log; exit 1; }
cd $R && python tools/pmc_table.py $O/a/*counter_collection.csv $O/b/*counter_collection.csv --out $O/table.json > $O/table.txt 2>&1; cat $O/table.txt | head -40
