# tile-config experiments: DNN_HIP_CFG / DNN_HIP_CFG16="K:cfg,..." override the chooser for the
# layer with that K (fp32 / fp16 plans); writes gpurun_out/cfg_<tag>.log
mkdir -p gpurun_out
run() { DNN_HIP_CFG16="$1" timeout -k 10 200 python bench.py --precision fp16 --steps 20 --warmup 5 --no-cpu --no-latency --no-e2e --no-fp16 --no-unfused --kernels > gpurun_out/cfg_$2.log 2>&1 || exit 1; }
run "" f16base
run "9216:7,4608:7" f16ns3
run "9216:8,4608:8" f16ns4
echo DONE
