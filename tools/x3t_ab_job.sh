# A/B of x3 tile-kernel variants in one call: ARMS="ENV=V ENV=V ..." -- the tile tests under each
# arm, then one bench per arm and the first arm again (per-kernel ms of conv1-conv3)
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/x3t; mkdir -p $O; cd $R
for a in $ARMS; do
env $a timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "x3_tile or yolo" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
echo "$a $(tail -1 $O/pytest.log)"
done
F="--steps 30 --warmup 5 --no-cpu --no-latency --no-fp16 --no-unfused --no-e2e --kernels"
for a in $ARMS ${ARMS%% *}; do
env $a timeout -k 10 120 python bench.py $F > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
tail -1 $O/b.log | python -c "import json,sys;d=json.loads(sys.stdin.read());k=d['kernels'];print('$a', d['value'], {n:v['ms'] for n,v in k.items() if n in ('conv1.patch','conv1.gemm','conv2.gemm','conv3.gemm')})"
done
