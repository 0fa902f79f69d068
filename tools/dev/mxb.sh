cd tools/micro
for f in "box2.0" "box1.0" "p5.0" "h5 3x3s2" "p4.0" "p5 c3k 3x3 64-64" ; do
  MX_TRACE=0 timeout -k 5 60 ./mx_bench "$f" 32 || exit 1
done
