set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --sampler napsac --steps 20 --warmup 3 --cpu-seconds 3 > gpurun_out/nap_bench.json 2> gpurun_out/nap_bench.err; rc=$?; cat gpurun_out/nap_bench.json; tail -3 gpurun_out/nap_bench.err; exit $rc
