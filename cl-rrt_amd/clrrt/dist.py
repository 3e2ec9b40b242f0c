"""Multi-GPU round exchange: samples shard by rank, accepted-node records are
all-gathered after every round and appended by every rank in global sample order, so the trees stay
identical.  One process per GPU; backend "nccl" (RCCL over xGMI) on the GPU box, "gloo" in the CPU
tests.

Record = clrrt_node (160 bytes, include/clrrt.h); rank r holds the records of its contiguous slice of
the round's samples, in sample order, so concatenating the slices in rank order IS global order.
"""
import torch
import torch.distributed as dist

REC_BYTES = 160
GOAL_OFFSET = 140  # clrrt_node.goal (int32)


def exchange_round(out_buf, n_local, elapsed_ms, group=None):
    """All-gather one round.

    out_buf: uint8 tensor (cap, 160) whose first n_local rows are this rank's records.
    elapsed_ms: this rank's elapsed query time (the horizon test uses the maximum over ranks, so
    every rank stops after the same round).
    Returns (records (total, 160) uint8 in global sample order, counts per rank, first row of this
    rank's records, max elapsed ms).
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = out_buf.device
    # gloo moves host tensors only: stage device buffers through the host (CPU rehearsal of the path)
    host = dist.get_backend(group) == "gloo" and dev.type != "cpu"
    cdev = torch.device("cpu") if host else dev
    meta = torch.tensor([float(n_local), float(elapsed_ms)], dtype=torch.float64, device=cdev)
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    counts = [int(m[0].item()) for m in metas]
    t_max = max(float(m[1].item()) for m in metas)
    src = out_buf.to(cdev) if host else out_buf.contiguous()
    bufs = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(bufs, src, group=group)
    parts = [bufs[r][:counts[r]] for r in range(world)]
    cat = torch.cat(parts, 0).contiguous() if sum(counts) else src[:0]
    if host:
        cat = cat.to(dev)
    return cat, counts, sum(counts[:rank]), t_max


def goal_count(records):
    """Appended nodes with goalReached set (feasible paths) among the records."""
    if records.shape[0] == 0:
        return 0
    return int(records[:, GOAL_OFFSET:GOAL_OFFSET + 4].contiguous().view(torch.int32).sum().item())


def shard(n_total, world, rank):
    """Contiguous slice [first, first + count) of a round's samples handled by `rank`."""
    per = n_total // world
    return rank * per, per


def fetch_path_rows(planner, rank, group=None):
    """Complete the committed path's trajectories across ranks (config 5 with N > 1).

    clrrt_path_commit copies the rows of nodes this rank owns and zero-fills the others; the path
    (a few nodes, a few thousand rows) is all-gathered and every node takes its rows from its owner,
    so every rank ends up with the same committed path.  Returns the number of rows moved."""
    import numpy as np
    nodes, rows = planner.path_download()
    if len(nodes) == 0:
        return 0
    world = dist.get_world_size(group)
    cdev = torch.device("cpu") if dist.get_backend(group) == "gloo" else torch.device("cuda", torch.cuda.current_device())
    t = torch.from_numpy(np.ascontiguousarray(rows)).to(cdev)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    parts = [p.cpu().numpy() for p in parts]
    fixed = rows.copy()
    moved = 0
    for nd in nodes:
        if nd.owner != rank:
            a, b = nd.row_offset, nd.row_offset + nd.nrows
            fixed[a:b] = parts[nd.owner][a:b]
            moved += nd.nrows
    if moved:
        planner.path_load(nodes, fixed)
    return moved
