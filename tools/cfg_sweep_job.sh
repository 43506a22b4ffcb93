# tile-config experiments: DNN_HIP_CFG / DNN_HIP_CFG16="K:cfg,..." override the chooser for the
# layer with that K (fp32 / fp16 plans); writes gpurun_out/cfg_<tag>.log
mkdir -p gpurun_out
run() { DNN_HIP_CFG="$1" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-latency --no-e2e --no-fp16 --no-unfused --kernels > gpurun_out/cfg_$2.log 2>&1 || exit 1; }
run "9216:9,4608:9,2304:9" c567_128x256
run "9216:11,4608:11,2304:9" c67_128x512
run "9216:11,4608:11,2304:11" c567_128x512
echo DONE
