set -u
mkdir -p gpurun_out/r02a
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02a/head -o head -- python3 bench.py --headline-only > gpurun_out/r02a/head.log 2>&1; rc=$?
echo "== prof headline rc=$rc"; tail -2 gpurun_out/r02a/head.log; [ $rc -eq 0 ] || exit $rc
