"""The multi-GPU round protocol through libclrrt with two ranks — GPU (both processes share device 0; the
gloo backend stages the exchange through the host, the rest is the path bench.py runs over RCCL).

Each rank evaluates its contiguous half of every round's 2B samples with clrrt_round_prefetch /
clrrt_round_eval, the records are exchanged with clrrt.dist.RoundExchange (one count-prefixed
all-gather), and clrrt_round_commit appends the union in global sample order; trajectory rows stay on
the rank that grew them (`owner`).  After 4 rounds at B = 4096 per rank each rank commits the best path
(extractBestPath, rrtplanner.cpp:318-368) and completes its rows with clrrt.dist.fetch_path_rows.

Checks against ONE process expanding the same stream with 2B samples per round (SURVEY.md §8(e):
sharding by samples does not change the result): identical node headers on both ranks (owner and
row_offset aside), the rows of every node equal on its owner, and the committed path's rows equal on
both ranks.
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD, B, ROUNDS, SEED = 2, 4096, 4, 17
HDR = 148  # clrrt_node bytes before owner / row_offset


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _planner(world=WORLD):
    import clrrt
    from clrrt import abi, scenes
    # (the single-process reference runs world x B samples per round: its conservative arena check wants room for
    # 2 full-horizon rows per sample of a round + its deferred samples)
    pl = clrrt.Planner(clrrt.default_params(collision_mode=abi.CLRRT_COLLISION_OBB), device=0, max_nodes=1 << 18,
                       max_rows=(1 << 25) * max(1, world // 2), max_batch=world * B)
    pl.set_obstacles(scenes.urban_scene(200))
    pl.tree_init()
    return pl


def _worker(rank, port, out_dir):
    sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    import clrrt
    from clrrt import abi
    from clrrt import dist as cdist
    pl = _planner()
    pl.set_rank(rank)
    pl.set_stream(torch.cuda.current_stream().cuda_stream)
    rx = cdist.RoundExchange(2 * B, "cuda", first_bound=256)
    rng = clrrt.Rng(SEED)
    first, count = cdist.shard(WORLD * B, WORLD, rank)
    nxt = rng.draw_samples(pl.params, WORLD * B)
    for _ in range(ROUNDS):
        cur, nxt = nxt, rng.draw_samples(pl.params, WORLD * B)
        mine = (abi.Sample * count).from_buffer(cur, first * 24)
        pl.round_prefetch((abi.Sample * count).from_buffer(nxt, first * 24))
        n_local = pl.round_eval(mine, rx.records_ptr())
        cat, counts, my_first, _ = rx.exchange(n_local, 0.0)
        pl.round_commit(cat.data_ptr() if cat.shape[0] else 0, cat.shape[0], my_first, counts[rank])
    raw = np.frombuffer(bytes(pl.nodes_raw()), dtype=np.uint8).reshape(-1, 160)
    g = pl.nodes()
    own = np.nonzero(g["owner"] == rank)[0]
    rows = [pl.rows(int(g["row_offset"][i]), int(g["nrows"][i])) for i in own]
    ids, _, _ = pl.extract_best_path()
    pl.path_commit(ids)
    moved = cdist.fetch_path_rows(pl, rank)
    _, prow = pl.path_download()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), hdr=raw[:, :HDR], own=own,
             rows=np.concatenate(rows) if rows else np.zeros((0, 10)), ids=np.array(ids, dtype=np.int64),
             prow=prow, moved=moved, second=rx.second_gathers)
    dist.barrier()
    dist.destroy_process_group()
    pl.close()


def test_two_ranks_on_one_gpu_match_single_process(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    import clrrt
    pl = _planner()
    st = pl.expand(clrrt.Rng(SEED), n_iters=ROUNDS * WORLD * B, mode=clrrt.CLRRT_MODE_BATCH, batch=WORLD * B)
    assert st["rounds"] == ROUNDS
    ref_raw = np.frombuffer(bytes(pl.nodes_raw()), dtype=np.uint8).reshape(-1, 160)
    g = pl.nodes()
    ranks = [np.load(tmp_path / f"rank{r}.npz") for r in range(WORLD)]
    print(f"2 ranks x {B} samples x {ROUNDS} rounds: {ref_raw.shape[0]} nodes; owned "
          f"{[len(r['own']) for r in ranks]}; path {len(ranks[0]['ids'])} nodes, rows moved "
          f"{[int(r['moved']) for r in ranks]}, second gathers {[int(r['second']) for r in ranks]}")
    assert ref_raw.shape[0] > 2000
    for r in ranks:
        assert np.array_equal(r["hdr"], ref_raw[:, :HDR])
    assert sum(len(r["own"]) for r in ranks) == ref_raw.shape[0]  # the root is owned by rank 0 only
    for rk, r in enumerate(ranks):
        want = [pl.rows(int(g["row_offset"][i]), int(g["nrows"][i])) for i in r["own"]]
        want = np.concatenate(want) if want else np.zeros((0, 10))
        assert np.array_equal(r["rows"].view(np.uint64), want.view(np.uint64)), rk
    ids, _, _ = pl.extract_best_path()
    pl.path_commit(ids)
    _, prow = pl.path_download()
    assert len(ids) >= 2
    for r in ranks:
        assert list(r["ids"]) == list(ids)
        assert np.array_equal(r["prow"].view(np.uint64), prow.view(np.uint64))
    assert sum(int(r["moved"]) for r in ranks) > 0  # the path crossed ranks
    pl.close()


# ---------------------------------------------------------------------------------------------------------
# The engine's own sharded rounds (clrrt_set_shards + clrrt.dist.ShardExchange): clrrt_expand runs every round
# on each rank -- its slice of the samples, the lag-1 / lag-2 pipelines, deferred samples -- and the exchange
# hook all-gathers the records; the same code path as one GPU.
SHARD_CASES = [  # (ranks, samples per round over all ranks, defer_steps, nn_lag, rounds)
    (2, 2 * B, 0, 1, 4),
    (2, 2 * B, 64, 2, 6),
    (2, 2 * B - 7, 48, 1, 4),   # uneven slices (shard_slice), deferred samples
    (4, 4 * B, 128, 2, 5),      # four ranks, the cfg3 bench's defer_steps
    (4, 4 * B - 5, 64, 1, 4),
    # cfg4's split rehearsed on one GPU (verdict r05 item 1): 8 ranks, the bench's G = 16384 per round strongly
    # split (2048 samples per rank), defer_steps 128, the lag-2 pipeline, 200 obstacles
    (8, 16384, 128, 2, 5),
]


def _shard_worker(rank, port, out_dir, world, G, T, lag, rounds, fail_rank=-1, fail_round=0, fail_opt="fail_at_round"):
    sys.path.insert(0, os.path.join(ROOT, "cl-rrt_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import clrrt
    from clrrt import dist as cdist
    pl = _planner(world)
    pl.set_option("defer_steps", T)
    pl.set_option("nn_lag", lag)
    pl.set_stream(torch.cuda.current_stream().cuda_stream)
    ex = cdist.ShardExchange(pl, cdist.exchange_capacity(-(-G // world), T), "cuda", slice_size=-(-G // world))
    if rank == fail_rank:
        pl.set_option(fail_opt, fail_round)
    err = ""
    try:
        st = pl.expand(clrrt.Rng(SEED), n_iters=rounds * G, mode=clrrt.CLRRT_MODE_BATCH, batch=G)
    except clrrt.ClrrtError as e:
        st, err = None, str(e)
    if st is None:
        np.savez(os.path.join(out_dir, f"shard{rank}.npz"), err=err, ex_rounds=ex.rounds)
        dist.destroy_process_group()
        pl.close()
        return
    raw = np.frombuffer(bytes(pl.nodes_raw()), dtype=np.uint8).reshape(-1, 160)
    g = pl.nodes()
    own = np.nonzero(g["owner"] == rank)[0]
    rows = [pl.rows(int(g["row_offset"][i]), int(g["nrows"][i])) for i in own]
    np.savez(os.path.join(out_dir, f"shard{rank}.npz"), hdr=raw[:, :HDR], own=own,
             rows=np.concatenate(rows) if rows else np.zeros((0, 10)), rounds=st["rounds"], it=st["iterations"],
             goals=st["goal_nodes_added"], deferred=st["deferred"], ex_rounds=ex.rounds,
             collectives=ex.collectives, closing=ex.closing, err=err)
    dist.barrier()
    dist.destroy_process_group()
    pl.close()


@pytest.mark.parametrize("world,G,T,lag,rounds", SHARD_CASES)
def test_sharded_expand_matches_single_process(tmp_path, world, G, T, lag, rounds):
    """Two or four ranks sharing GPU 0 run clrrt_expand with the exchange hook; every tree equals ONE process
    expanding the same stream with G samples per round (same defer_steps): headers bit for bit, every node's rows
    on its owner, the iteration count and the goal nodes appended (every rank's).  One collective
    per exchange (the gather bound starts at the slice size, so no round needs a second gather)."""
    import torch.multiprocessing as mp
    mp.spawn(_shard_worker, args=(_free_port(), str(tmp_path), world, G, T, lag, rounds), nprocs=world, join=True)
    import clrrt
    pl = _planner(world)
    pl.set_option("defer_steps", T)
    pl.set_option("nn_lag", lag)
    st = pl.expand(clrrt.Rng(SEED), n_iters=rounds * G, mode=clrrt.CLRRT_MODE_BATCH, batch=G)
    assert st["rounds"] == rounds and (T == 0 or st["deferred"] > 0), st
    ref_raw = np.frombuffer(bytes(pl.nodes_raw()), dtype=np.uint8).reshape(-1, 160)
    g = pl.nodes()
    ranks = [np.load(tmp_path / f"shard{r}.npz") for r in range(world)]
    print(f"sharded x{world} G={G} T={T} lag {lag}: {ref_raw.shape[0]} nodes; owned {[len(r['own']) for r in ranks]}; "
          f"deferred {[int(r['deferred']) for r in ranks]} (single {st['deferred']}); exchanges "
          f"{[int(r['ex_rounds']) for r in ranks]}, collectives {[int(r['collectives']) for r in ranks]}")
    assert ref_raw.shape[0] > 2000
    for r in ranks:
        assert str(r["err"]) == ""
        assert np.array_equal(r["hdr"], ref_raw[:, :HDR])
        assert int(r["rounds"]) == rounds and int(r["it"]) == rounds * G
        assert int(r["goals"]) == st["goal_nodes_added"]
        assert int(r["collectives"]) == int(r["ex_rounds"]) >= rounds
        assert int(r["closing"]) == 1  # one closing exchange per expansion
    assert sum(int(r["deferred"]) for r in ranks) == st["deferred"]
    assert sum(len(r["own"]) for r in ranks) == ref_raw.shape[0]
    for rk, r in enumerate(ranks):
        want = [pl.rows(int(g["row_offset"][i]), int(g["nrows"][i])) for i in r["own"]]
        want = np.concatenate(want) if want else np.zeros((0, 10))
        assert np.array_equal(r["rows"].view(np.uint64), want.view(np.uint64)), rk
    pl.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("fail_round", [1, 3])
def test_sharded_failure_is_collective(tmp_path, fail_round):
    """A failure on one rank only (option fail_at_round: its commit of that round fails, after the deferred-sample
    bookkeeping) ends the expansion on every rank with an error, instead of leaving the others waiting in the
    round's all-gather: the failed rank joins the exchange the others make with an error flag."""
    import torch.multiprocessing as mp
    mp.spawn(_shard_worker, args=(_free_port(), str(tmp_path), 2, 2 * B, 64, 2, 6, 1, fail_round), nprocs=2,
             join=True)
    r0, r1 = (np.load(tmp_path / f"shard{r}.npz") for r in range(2))
    print(f"fail at round {fail_round}: rank 0 '{r0['err']}', rank 1 '{r1['err']}', exchanges "
          f"{int(r0['ex_rounds'])} / {int(r1['ex_rounds'])}")
    assert "injected failure" in str(r1["err"])
    assert "rank(s) failed" in str(r0["err"])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("T,lag", [(0, 1), (0, 2), (64, 2)])
def test_sharded_failure_after_last_exchange_is_collective(tmp_path, T, lag):
    """a rank that fails AFTER the last round's exchange (option fail_after_exchange: the work that
    follows the exchange fails) -- with defer_steps 0 no drain exchange follows -- still ends the expansion on every
    rank with an error: every sharded expansion closes with one exchange that carries the failure, so no rank waits
    in a collective the failed rank never joins and no rank reports success beside a failed one."""
    import torch.multiprocessing as mp
    rounds = 4
    mp.spawn(_shard_worker, args=(_free_port(), str(tmp_path), 2, 2 * B, T, lag, rounds, 1, rounds,
                                  "fail_after_exchange"), nprocs=2, join=True)
    r0, r1 = (np.load(tmp_path / f"shard{r}.npz") for r in range(2))
    print(f"T={T} lag {lag}, fail after exchange {rounds}: rank 0 '{r0['err']}', rank 1 '{r1['err']}', exchanges "
          f"{int(r0['ex_rounds'])} / {int(r1['ex_rounds'])}")
    assert "injected failure" in str(r1["err"])
    assert "rank(s) failed" in str(r0["err"])


@pytest.mark.timeout(300)
def test_deferred_error_then_flush(tmp_path):
    """An expansion with deferred samples that fails mid-way (fault injection) leaves no suspended chains behind:
    the rows flush, a fresh tree and a new expansion afterwards work and grow the tree a fresh context grows."""
    import clrrt
    trees = []
    for inject in (True, False):
        pl = _planner(1)
        pl.set_option("defer_steps", 32)
        if inject:
            pl.set_option("fail_at_round", 3)
            with pytest.raises(clrrt.ClrrtError, match="injected failure"):
                pl.expand(clrrt.Rng(5), n_iters=6 * B, mode=clrrt.CLRRT_MODE_BATCH, batch=B)
            pl.rows_flush()
            pl.tree_init()
        st = pl.expand(clrrt.Rng(SEED), n_iters=4 * B, mode=clrrt.CLRRT_MODE_BATCH, batch=B)
        assert st["deferred"] > 0
        n, nr = pl.size()
        trees.append((bytes(pl.nodes_raw()), pl.rows(0, nr).tobytes()))
        pl.close()
    assert trees[0] == trees[1]
