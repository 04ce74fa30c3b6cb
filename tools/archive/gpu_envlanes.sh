set -o pipefail
for l in 16 32 64; do for w in 1 4; do
FFMP_ENV_LANES=$l FFMP_ENV_WAVES=$w timeout -k 10 120 python3 tools/env_kernel_breakdown.py --preset C2 --envs 4096 base 2>&1 | grep 'env kernel' | sed "s/^/lanes=$l waves=$w /" || exit 1
done; done
