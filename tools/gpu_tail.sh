set -o pipefail
for v in p1 p2 default p8; do
  if [ $v == default ]; then L=zraytrace_amd/libzrt.so; else L=build/variants/$v/libzrt.so; fi
  echo "== $v"; ZRT_LIB=$L timeout -k 10 300 python tools/tail_probe.py 8 2 2048 2048 1024 20 short || exit 1
done
