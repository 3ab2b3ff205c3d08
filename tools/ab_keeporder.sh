set -o pipefail
for L in base keeporder base keeporder; do
  echo "== $L"; FLASHSDF_LIB=$PWD/abr/lib_$L.so timeout -k 10 120 python tools/descend_probe.py --frames 7 2>&1 | grep loop || exit 1
done
