set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh r3c tests/test_gpu_sharded_run.py tests/test_gpu_napsac_lo.py tests/test_gpu_cpp_consumer.py || exit $?
for e in fundamental essential homography; do
  timeout -k 10 300 python bench.py --estimator $e --cpu-seconds 3 > gpurun_out/r3c_bench_$e.json 2> gpurun_out/r3c_bench_$e.err || exit $?
done
