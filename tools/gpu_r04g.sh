set -u
O=gpurun_out/r04g; mkdir -p $O
for L in conv3 deconv1 deconv2 conv2; do
  ICLR17_LIB=build/st/libiclr17.so timeout -k 10 120 python tools/k5_stamps.py $L > $O/st_$L.log 2>&1 || { cat $O/st_$L.log; exit 1; }
  head -8 $O/st_$L.log
done
