set -o pipefail
timeout -k 10 120 ./tools/cr_bench 1 112 5 | head -1 && \
for p in 2 3 278; do timeout -k 10 120 ./tools/cr_bench $p 112 10 2>&1 | grep -v top_phase | grep -v factor_check || exit 1; done
