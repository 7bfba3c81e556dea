export TMPDIR=/tmp; mkdir -p gpurun_out/r03m
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03m/tests.log 2>&1 || exit 1
R=3 timeout -k 10 600 bash tools/ab_libs.sh gpurun_out/r03m/ab ab_old/b0.so iclr_17_compression_amd/libiclr17.so || exit 1
