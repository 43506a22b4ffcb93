# bench value with events around every kernel (--kernels) vs around the dominant kernel only
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/tab; mkdir -p $O; cd $R
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "timing_api" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
F="--steps 40 --warmup 5 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e"
for k in "" "--kernels" "" "--kernels"; do
timeout -k 10 120 python bench.py $F $k > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
tail -1 $O/b.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$k', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['conv_mfma'])"
done
