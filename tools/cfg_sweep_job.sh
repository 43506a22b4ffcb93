# tile-config experiments: DNN_HIP_CFG="K:cfg,..." overrides the chooser for the layer with that K
mkdir -p gpurun_out
run() { DNN_HIP_CFG="$1" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-latency --no-e2e --no-fp16 --no-unfused --kernels > gpurun_out/cfg_$2.log 2>&1 || exit 1; }
run "" base
run "288:9" c2_128x64
run "288:9,576:9" c23_128x64x
echo DONE
