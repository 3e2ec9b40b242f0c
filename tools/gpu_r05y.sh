# Round 5: the appended-node search in place order (option nn_delta_place) -- the GPU suite's list / pipelined / full-size
# tests, then the cfg3 bench with the option on / off (x2, alternating) and a kernel trace of the round's critical path.
set -e
tag=${1:-r05y}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_parity.py tests/test_ref_tree.py tests/test_dist_gpu.py \
  -m gpu -x -v --timeout 900 --timeout-method thread > $out/gpu_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-cpu --no-exact --no-sync --opt nn_delta_place=1 > $out/bench_on$i.json 2> $out/bench_on$i.err
  timeout -k 10 300 python3 -u bench.py --no-cpu --no-exact --no-sync --opt nn_delta_place=0 > $out/bench_off$i.json 2> $out/bench_off$i.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tr -o p \
  -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu --no-exact --no-sync > $out/bench_tr.json 2> $out/bench_tr.err
python3 tools/round_crit.py $out/tr/p_kernel_trace.csv > $out/round_crit.txt
python3 - $out/tr/p_kernel_trace.csv >> $out/round_crit.txt <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    d[r["Kernel_Name"][:48]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda x: -sum(x[1]))[:10]:
    v.sort()
    print(f"{k:48s} n {len(v):5d} median {v[len(v)//2]:8.1f} us p90 {v[int(len(v)*.9)]:8.1f} us")
PY
rm -f $out/tr/p_kernel_trace.csv
echo done
