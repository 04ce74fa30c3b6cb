set -o pipefail
for rep in 1 2 3; do
  for v in "1 1 1" "1 0 0" "0 0 0" "0 1 0"; do
    timeout -k 10 120 python tools/ring_variants.py $v 2>&1 | grep "^pair=" || exit 1
  done
done
