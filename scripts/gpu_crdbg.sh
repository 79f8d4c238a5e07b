set -o pipefail
for p in 1 2 3 278; do timeout -k 10 120 ./tools/cr_bench $p 112 10 2>&1 || exit 1; done
