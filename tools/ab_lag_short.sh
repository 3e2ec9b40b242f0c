# A/B of nn_lag 1 vs 2 on the short-query configurations (cfg2, cfg5: 200 ms queries), two reps each.
# Usage (GPU box, repo root): bash tools/ab_lag_short.sh
set -e
out=gpurun_out/ab_cfg; mkdir -p $out
for rep in 1 2; do for cfg in cfg2 cfg5; do for lag in 1 2; do
  timeout -k 10 150 python3 -u bench.py --config $cfg --steps 5 --warmup 1 --no-cpu --no-exact --opt nn_lag=$lag > $out/${cfg}_${lag}_${rep}.json 2>/dev/null
  python3 -c "import json; d=json.loads(open('$out/${cfg}_${lag}_${rep}.json').read().strip().splitlines()[-1]); print('$cfg lag $lag rep $rep', round(d['value']/1e6,4))"
done; done; done
