# Kernel traces of short cfg3 bench runs (default options, then each KEY=VALUE given) and their round gaps.
# Usage (GPU box, repo root): bash tools/gap_trace.sh <out_dir> [KEY=VALUE ...]
set -e
out=${1:-gpurun_out/gaps}
shift || true
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p $out
i=0
for opt in "" "$@"; do
  i=$((i+1))
  extra=""
  [ -n "$opt" ] && extra="--opt $opt"
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/t$i -o p \
    -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu --no-exact $extra > $out/t$i.json 2> $out/t$i.err
  echo "variant $i [$opt]: $(python3 -c "import json; d=json.loads(open('$out/t$i.json').read().strip().splitlines()[-1]); print(round(d['value']))")"
  python3 tools/round_gaps.py $out/t$i/p_kernel_trace.csv > $out/gaps$i.txt
  grep -E "gaps, mean|query" $out/gaps$i.txt | head -4
  rm -f $out/t$i/p_kernel_trace.csv
done
