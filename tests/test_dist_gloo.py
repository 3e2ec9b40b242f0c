"""World-size-2 test of the multi-GPU round protocol on CPU (gloo): every rank evaluates its slice of
each round's samples against the frozen tree, the accepted-node records are exchanged with
clrrt.dist.RoundExchange (the count-prefixed all-gather bench.py runs over RCCL), and every rank appends the union in
global sample order.  The CPU oracle stands in for the GPU evaluator (test infrastructure only).

Checks: both ranks end with the identical tree, and it equals the single-process BATCH expansion
(sharding by samples does not change the result).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

WORLD, PER_RANK, ROUNDS, SEED = 2, 24, 4, 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle(obs):
    from clrrt import abi
    from oracle_binding import Oracle
    o = Oracle(abi.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), obs)
    Oracle.srand(SEED)
    o.init_tree()
    return o


def _worker(rank, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from clrrt import abi, scenes
    from clrrt import dist as cdist
    obs = scenes.urban_scene(200)
    o = _oracle(obs)
    rx = cdist.RoundExchange(2 * PER_RANK, "cpu", first_bound=4)  # small bound: exercises the second gather
    for _ in range(ROUNDS):
        xy, ex = o.draw_samples(WORLD * PER_RANK)   # the single glibc stream, drawn by every rank
        first, count = cdist.shard(WORLD * PER_RANK, WORLD, rank)
        recs = []
        for j in range(first, first + count):         # frozen tree: nothing appended yet
            recs += o.eval_iteration(xy[j][0], xy[j][1], ex[j], stable=True)
        raw = bytes((abi.Node * len(recs))(*recs)) if recs else b""
        rx.records().zero_()
        if raw:
            rx.records()[:len(recs)] = torch.frombuffer(bytearray(raw), dtype=torch.uint8).view(len(recs), cdist.REC_BYTES)
        cat, counts, my_first, t_max = rx.exchange(len(recs), 10.0 * (rank + 1))
        assert my_first == sum(counts[:rank]) and cat.shape[0] == sum(counts) and t_max == 10.0 * WORLD
        # commit in global order: goal-biased records name the record before them as parent
        base = o.size()
        cur = list(o.nodes_raw())
        new = (abi.Node * cat.shape[0]).from_buffer_copy(cat.numpy().tobytes()) if cat.shape[0] else []
        for k, nd in enumerate(new):
            if nd.parent == abi.CLRRT_PARENT_PREV:
                nd.parent = base + k - 1
            cur.append(nd)
        o.load_tree((abi.Node * len(cur))(*cur))
    assert rx.second_gathers >= 1  # the first round's counts exceeded the initial bound of 4
    n = o.nodes()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), state=n["state"], parent=n["parent"], goal=n["goal"],
             nrows=n["nrows"], costE=n["costE"], costS=n["costS"])
    dist.destroy_process_group()


def test_two_rank_round_exchange_matches_single_process(tmp_path):
    from clrrt import scenes
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    r0 = np.load(tmp_path / "rank0.npz")
    r1 = np.load(tmp_path / "rank1.npz")
    for k in r0.files:
        assert np.array_equal(r0[k], r1[k]), k
    ref = _oracle(scenes.urban_scene(200))
    ref.expand_batch(ROUNDS * WORLD * PER_RANK, WORLD * PER_RANK, stable=True)
    n = ref.nodes()
    assert len(n["parent"]) == len(r0["parent"]) > 1
    # (nrows is not compared: the oracle's load_tree keeps headers only, not trajectories)
    for k in ("state", "parent", "goal", "costE", "costS"):
        assert np.array_equal(np.asarray(n[k]), r0[k]), k


def test_shard_slices_cover_the_round():
    from clrrt import dist as cdist
    for world in (1, 2, 4, 8):
        seen = []
        for r in range(world):
            first, count = cdist.shard(16384 * world, world, r)
            seen += list(range(first, first + count))
        assert seen == list(range(16384 * world))


class _PathHolder:
    """Stands in for clrrt.Planner's committed-path entries (path_download / path_load)."""

    def __init__(self, nodes, rows):
        self.nodes, self.rows = nodes, rows

    def path_download(self):
        return self.nodes, self.rows.copy()

    def path_load(self, nodes, rows):
        self.nodes, self.rows = nodes, np.array(rows)


def _path_worker(rank, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from clrrt import abi
    from clrrt import dist as cdist
    owners, nrows = [0, 1, 1, 0], [1, 3, 2, 4]
    nodes = (abi.Node * 4)()
    full = np.arange(sum(nrows) * 10, dtype=np.float64).reshape(-1, 10) - 7.0
    rows = np.zeros_like(full)
    off = 0
    for i in range(4):
        nodes[i].owner, nodes[i].nrows, nodes[i].row_offset = owners[i], nrows[i], off
        if owners[i] == rank:  # what clrrt_path_commit leaves: own rows copied, the others zero
            rows[off:off + nrows[i]] = full[off:off + nrows[i]]
        off += nrows[i]
    h = _PathHolder(nodes, rows)
    moved = cdist.fetch_path_rows(h, rank)
    np.savez(os.path.join(out_dir, f"path{rank}.npz"), rows=h.rows, full=full, moved=moved)
    dist.destroy_process_group()


def test_two_rank_committed_path_rows_fetch(tmp_path):
    """Config 5 on N GPUs: every rank completes the committed path with the rows held by their owners."""
    mp.spawn(_path_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    for r in range(WORLD):
        d = np.load(tmp_path / f"path{r}.npz")
        assert np.array_equal(d["rows"], d["full"])
    assert int(np.load(tmp_path / "path0.npz")["moved"]) == 5 and int(np.load(tmp_path / "path1.npz")["moved"]) == 5
