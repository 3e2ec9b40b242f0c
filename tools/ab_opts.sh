# A/B of engine options on the cfg3 bench (results never depend on them): each variant twice, interleaved.
# Usage (GPU box, repo root): bash tools/ab_opts.sh <out_dir> "<opts A>" "<opts B>" ...   ("" = defaults)
# opts: space-separated KEY=VALUE (bench.py --opt); LIB=<path> runs that variant with another build of
# libclrrt (CLRRT_LIB).  Prints value (M nodes/s) per run.
set -e
out=$1; shift
mkdir -p $out
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    args=""
    lib=""
    for kv in $v; do
      case $kv in LIB=*) lib=${kv#LIB=} ;; *) args="$args --opt $kv" ;; esac
    done
    CLRRT_LIB=$lib timeout -k 10 150 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-exact $args > $out/v${i}_r$rep.json 2> $out/v${i}_r$rep.err
    python3 -c "import json,sys; d=json.load(open('$out/v${i}_r$rep.json')); print('variant $i [$v] rep $rep:', round(d['value']/1e6,4), 'M nodes/s, roll ms/launch', round(d.get('kernel_ms',{}).get('rollout',0)/max(1,d.get('kernel_launches',{}).get('rollout',1)),3) if isinstance(d.get('kernel_ms'),dict) else '')"
  done
done
