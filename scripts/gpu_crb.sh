set -o pipefail
for p in 1 278; do timeout -k 10 120 ./tools/cr_bench $p 112 10 2>&1 | grep -v factor_check || exit 1; done
