set -o pipefail
mkdir -p gpurun_out
for bl in 8 4; do
SQLM_TILE_BL=$bl timeout -k 10 300 python -u scripts/tile_prof.py > gpurun_out/tileprof_$bl.json 2>&1 || { tail -5 gpurun_out/tileprof_$bl.json; exit 1; }
echo BL $bl; cat gpurun_out/tileprof_$bl.json
done
