# x3 conv: parity tests, fp32 bench line with per-kernel times, SQ bank-conflict pass
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/x3q; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread -k "x3" > $O/pytest.log 2>&1 || { grep -E "err|PASS|FAIL|Error" $O/pytest.log | tail -30; exit 1; }
grep -E "normwise|passed|failed" $O/pytest.log | tail -8
F="--steps 20 --warmup 3 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels"
timeout -k 10 120 python bench.py $F > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernels'];print(d['value'], {n:(v['ms'],v['tflops']) for n,v in k.items() if n in ('pool5','conv6.gemm','conv7.gemm')})"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/b -o b --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
cd $R && python tools/pmc_table.py $O/b/*counter_collection.csv > $O/table.txt 2>&1; grep -E "kernel|conv6|conv7" $O/table.txt
