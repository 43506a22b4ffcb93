export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread -k "fp16_detections or postprocess" > gpurun_out/pytest_f16det.log 2>&1 || { tail -40 gpurun_out/pytest_f16det.log; exit 1; }
grep "fp16 detections" gpurun_out/pytest_f16det.log; tail -2 gpurun_out/pytest_f16det.log
