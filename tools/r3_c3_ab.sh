set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/match_pmc.sh m8 || exit 1
for n in c3base c3nw2 c3nw2t512 c3nw1 c3base; do
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 120 python3 tools/match_time.py > gpurun_out/mt_c3_$n.json 2>&1 || { echo "$n failed"; tail -5 gpurun_out/mt_c3_$n.json; exit 1; }
  echo "$n $(tail -1 gpurun_out/mt_c3_$n.json)"
done
