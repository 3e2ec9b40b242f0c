# Round 5: is k_select (1.7 ms in every other cfg3 round) held up by the walk's pending workgroups?  The persistent walk
# grid at 10 (default) / 8 / 6 waves per CU: bench value and the commit kernels' durations from a kernel trace.
set -e
tag=${1:-r05z}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
for w in 2560 2048 1536; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tr$w -o p \
    -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu --no-exact --no-sync --opt nn_walk_waves=$w > $out/bench_w$w.json 2> $out/bench_w$w.err
  python3 tools/round_crit.py $out/tr$w/p_kernel_trace.csv > $out/round_crit_w$w.txt
  python3 - $out/tr$w/p_kernel_trace.csv >> $out/round_crit_w$w.txt <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    d[r["Kernel_Name"][:48]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda x: -sum(x[1]))[:10]:
    v.sort()
    print(f"{k:48s} n {len(v):5d} median {v[len(v)//2]:8.1f} us p90 {v[int(len(v)*.9)]:8.1f} us")
PY
  rm -f $out/tr$w/p_kernel_trace.csv
done
echo done
