set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/tr5 -o run --output-format csv -- python3 tools/cfg5_split.py 5 > /dev/null 2> gpurun_out/tr5.err || exit $?
