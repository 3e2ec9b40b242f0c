"""Where the lists of a lag-2 round come from (rocprofv3 kernel trace of a cfg3 bench): for every gap between two
rollout kernels on the main stream, the appended-node merge (k_nn_merge_delta) that ended last before the next rollout
kernel, and before it on its stream the appended-node search (k_nn_partial), and on the walk streams the last main walk
grid, split launch and split merge that ended before that merge began.  Times in us after the rollout kernel's end.
Usage: python3 tools/list_crit.py <p_kernel_trace.csv[.gz]>"""
import bisect
import csv
import gzip
import statistics as S
import sys


def kname(n):
    if n.startswith("void clrrt::k_walk_search<"):
        return "walk_split" if n.split(",")[1].strip() == "true" else "walk_main"
    return n.split("(")[0].replace("void ", "").replace("clrrt::", "").split("<")[0]


def main(path):
    op = gzip.open if path.endswith(".gz") else open
    by = {}
    roll = []
    for r in csv.DictReader(op(path, "rt")):
        k = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"])
        n = kname(r["Kernel_Name"])
        if r["Kernel_Name"].startswith("void clrrt::k_roll_run<false, true, true>"):
            roll.append(k)
        by.setdefault(n, []).append(k)
    roll.sort()
    ends = {}
    for n, v in by.items():
        v.sort(key=lambda k: k[1])
        ends[n] = [k[1] for k in v]

    def last_before(n, t, stream=None, after=None):
        if n not in by:
            return None
        i = bisect.bisect_right(ends[n], t) - 1
        while i >= 0:
            k = by[n][i]
            if after is not None and k[1] < after:
                return None
            if stream is None or k[2] == stream:
                return k
            i -= 1
        return None

    res = {k: [] for k in ("walk_main_end", "split_start", "split_end", "wmerge_end", "partial_start", "partial_end",
                           "dmerge_end", "next_rollout")}
    for i in range(len(roll) - 1):
        t0, t1 = roll[i][1], roll[i + 1][0]
        if t1 - t0 > 20e6:
            continue
        d = last_before("k_nn_merge_delta", t1, after=roll[i][0])
        if not d:
            continue
        f = lambda t: (t - t0) / 1e3
        res["next_rollout"].append(f(t1))
        res["dmerge_end"].append(f(d[1]))
        p = last_before("k_nn_partial", d[0], stream=d[2], after=roll[i][0] - 5e6)
        if p:
            res["partial_start"].append(f(p[0]))
            res["partial_end"].append(f(p[1]))
        for n, a, b in (("k_walk_merge", None, "wmerge_end"), ("walk_split", "split_start", "split_end"),
                        ("walk_main", None, "walk_main_end")):
            k = last_before(n, p[0] if p else d[0], after=roll[i][0] - 15e6)
            if k:
                if a:
                    res[a].append(f(k[0]))
                res[b].append(f(k[1]))
    print("us after the rollout kernel's end (median / p10 / p90 over %d gaps):" % len(res["next_rollout"]))
    for k, v in res.items():
        if v:
            v = sorted(v)
            print("  %-14s %8.0f %8.0f %8.0f" % (k, S.median(v), v[len(v) // 10], v[9 * len(v) // 10]))


if __name__ == "__main__":
    main(sys.argv[1])
