# all GPU tests, then the default bench line: headline, latency (batch-1 latency plan) and its kernels
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/x3l; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "normwise|FAIL|Error|^E " $O/pytest.log | tail -30; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c "
import json,sys;d=json.loads(sys.stdin.read());l=d['latency_b1']
print('value', d['value'], 'roofline', d['roofline']['achieved'], d['roofline']['frac'])
print('latency', {k:l[k] for k in ('eager_ms','graph_ms','graph_device_ms','normwise_err_vs_batch_plan')})
print(l['kernel_ms'])
print('batch plan at b1', l['batch_plan_at_batch1']['graph_device_ms'])"
