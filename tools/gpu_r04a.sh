set -u
O=gpurun_out/r04a; mkdir -p $O; export TMPDIR=/tmp
export ICLR17_PARITY_OUT=$O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_operating_point.py "tests/test_gpu_parity.py::test_encoder_with_grad_matches_codec_forward" "tests/test_gpu_parity.py::test_encoder_matches_codec_forward" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python bench.py --mode kodak > $O/kodak.json 2> $O/kodak.err || { tail $O/kodak.err; exit 1; }
ICLR17_DIST_BACKEND=gloo timeout -k 10 200 python bench.py --mode kodak --gpus 2 > $O/kodak_2rank.json 2> $O/kodak_2rank.err || { tail $O/kodak_2rank.err; exit 1; }
timeout -k 10 200 python bench.py --mode encdec > $O/encdec_x6.json 2> $O/encdec_x6.err || { tail $O/encdec_x6.err; exit 1; }
timeout -k 10 200 python bench.py --mode encdec --precision bf16 > $O/encdec_bf16.json 2> $O/encdec_bf16.err || { tail $O/encdec_bf16.err; exit 1; }
for f in kodak kodak_2rank encdec_x6 encdec_bf16; do grep '^{' $O/$f.json | tail -1 | cut -c1-900; done
