# Round 5: the walk's overflow split fan-out (option nn_walk_chunks 16 / 32 / 64) against the cfg3 round's critical path
# (kernel traces + tools/round_crit.py) and the bench value.
set -e
tag=${1:-r05u}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
for ch in 16 32 64; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tr$ch -o p \
    -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu --no-exact --no-sync --opt nn_walk_chunks=$ch > $out/bench_ch$ch.json 2> $out/bench_ch$ch.err
  python3 tools/round_crit.py $out/tr$ch/p_kernel_trace.csv > $out/round_crit_ch$ch.txt
  python3 - $out/tr$ch/p_kernel_trace.csv >> $out/round_crit_ch$ch.txt <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    d[r["Kernel_Name"][:48]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda x: -sum(x[1]))[:6]:
    v.sort()
    print(f"{k:48s} n {len(v):5d} median {v[len(v)//2]:8.1f} us p90 {v[int(len(v)*.9)]:8.1f} us")
PY
  rm -f $out/tr$ch/p_kernel_trace.csv
done
echo done
