set -e
for cfg in "256 1 256" "128 1 256" "64 1 1024" "256 2 512"; do
  set -- $cfg
  timeout -k 10 200 python -u tools/quality_sweep.py --instance x1000 --T 10 60 --seeds 0 --moves $1 --wg-per-cu $2 --chains $3 --no-cpu --out gpurun_out/scan_$1_$2.json
done
