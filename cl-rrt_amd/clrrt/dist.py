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


class RoundExchange:
    """All-gather of one round's accepted-node records, count-prefixed.

    Row 0 of `buf` is a header (int64 record count, float64 elapsed query ms, int64 aux value summed over the
    ranks, float64[4] bounds of the rank's record positions); clrrt_round_eval writes
    this rank's records from row 1 on (`records_ptr`).  One all-gather moves header + the first `bound`
    record rows of every rank, so no count exchange (and no host sync) precedes the data; the headers
    are read back once afterwards -- the one host wait of a round: the engine appends the union, so it needs the
    counts (and the budget word, the bounds) on the host.
    `bound` starts at `first_bound` (the sharded expansion passes this rank's slice size: a round commits
    about 0.4 records per sample) and adapts to 1.25x the largest count seen; a round whose count exceeds it
    (rare) moves the excess with a second all-gather (`second_gathers`; `collectives` counts them all).
    gloo (CPU rehearsal of the path) stages device buffers through the host.
    """

    HDR = 56

    def __init__(self, cap_records, device, group=None, first_bound=1024):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.cap = int(cap_records)
        self.dev = torch.device(device)
        self.buf = torch.zeros((self.cap + 1, REC_BYTES), dtype=torch.uint8, device=self.dev)
        self.bound = min(self.cap, first_bound)
        self.host = dist.get_backend(group) == "gloo" and self.dev.type != "cpu"
        self.second_gathers = 0
        self.collectives = 0
        self.exchanges = 0

    def records_ptr(self):
        """Device address where this rank's clrrt_round_eval output goes (row 1 of the buffer)."""
        return self.buf.data_ptr() + REC_BYTES

    def records(self):
        return self.buf[1:]

    def _gather(self, t):
        self.collectives += 1
        src = t.cpu() if self.host else t.contiguous()
        parts = [torch.empty_like(src) for _ in range(self.world)]
        dist.all_gather(parts, src, group=self.group)
        return parts

    def exchange(self, n_local, elapsed_ms, aux=0, bbox=None, engine_stream=None):
        """Returns (records (total, 160) uint8 on the buffer's device in global sample order, counts
        per rank, first row of this rank's records, max elapsed ms over ranks); the sum of `aux` over the
        ranks is left in self.aux_sum and the union of the ranks' `bbox` (x0, y0, x1, y1) in self.bbox_all.

        engine_stream (a HIP stream handle): the stream the records were written on and the gathered records will
        be read on.  The gather is ordered after it and it after the gather by stream waits, not by the host;
        without one, torch's stream is synchronised before returning (the round API's callers)."""
        import numpy as np
        self.exchanges += 1
        cuda = self.dev.type == "cuda"
        ext = None
        if cuda and engine_stream:
            cur = torch.cuda.current_stream(self.dev)
            if int(engine_stream) != cur.cuda_stream:
                ext = torch.cuda.ExternalStream(int(engine_stream), device=self.dev)
                cur.wait_stream(ext)  # the records were written on the engine's stream
        hdr = np.zeros(self.HDR // 8, dtype=np.float64)
        hdr.view(np.int64)[0] = int(n_local)
        hdr[1] = float(elapsed_ms)
        hdr.view(np.int64)[2] = int(aux)
        hdr[3:7] = bbox if bbox is not None else (np.inf, np.inf, -np.inf, -np.inf)
        self.buf[0, :self.HDR].copy_(torch.from_numpy(hdr.view(np.uint8)))
        parts = self._gather(self.buf[:self.bound + 1])
        heads = torch.stack([q[0, :self.HDR] for q in parts]).cpu().numpy()
        counts = [int(c) for c in heads[:, :8].copy().view(np.int64)[:, 0]]
        t_max = float(heads[:, 8:16].copy().view(np.float64).max())
        self.aux_sum = int(heads[:, 16:24].copy().view(np.int64).sum())
        bb = heads[:, 24:56].copy().view(np.float64).reshape(-1, 4)
        self.bbox_all = (float(bb[:, 0].min()), float(bb[:, 1].min()), float(bb[:, 2].max()), float(bb[:, 3].max()))
        maxc = max(counts)
        extra = None
        if maxc > self.bound:
            # the excess rows of every rank (padded to the largest count) in a second collective
            self.second_gathers += 1
            extra = self._gather(self.buf[1 + self.bound:1 + maxc])
        pieces = []
        for r in range(self.world):
            c = counts[r]
            pieces.append(parts[r][1:1 + min(c, self.bound)])
            if c > self.bound:
                pieces.append(extra[r][:c - self.bound])
        self.bound = min(self.cap, max(self.bound, int(maxc * 1.25) + 64))
        total = sum(counts)
        cat = torch.cat(pieces, 0) if total else self.buf[1:1]
        if self.host and total:
            cat = cat.to(self.dev)
        cat = cat.contiguous()
        if cuda:
            if ext is not None:
                ext.wait_stream(torch.cuda.current_stream(self.dev))  # the engine reads the gathered records
            elif not engine_stream:
                # no engine stream named: the caller reads the records on a stream of its own choosing
                torch.cuda.current_stream(self.dev).synchronize()
        return cat, counts, sum(counts[:self.rank]), t_max


class ShardExchange:
    """The exchange hook of the engine's own sharded rounds (clrrt_set_shards): clrrt_expand runs every
    round -- this rank's slice of the samples, the lag-2 pipeline, deferred samples -- and calls back once
    per round with its records in `records_ptr()` (written on the engine's stream, which it does not wait for);
    the callback runs RoundExchange's count-prefixed all-gather (RCCL over xGMI with the nccl backend) ordered
    after the engine's stream by a stream wait, and hands the concatenation in rank order back, with the largest
    elapsed query time over the ranks (the engine's budget decision, identical on every rank) and the union of the
    ranks' position bounds; the engine's stream waits for the gather (no host synchronisation besides reading
    the headers).  Every sharded expansion ends with a closing exchange (no records) that carries any rank's
    failure.  One code path for 1 and N GPUs: with world 1 the engine appends its records itself."""

    def __init__(self, planner, cap_records, device, group=None, first_bound=None, slice_size=None):
        import traceback
        from . import EXCHANGE_FN
        if first_bound is None:
            # a round commits ~0.4 records per sample of the slice (2 at most): one slice's worth of rows covers the
            # first rounds without a second gather (then the bound follows the counts seen)
            first_bound = int(slice_size) + 64 if slice_size else 1024
        self.rx = RoundExchange(cap_records, device, group, first_bound)
        self.rank, self.world = self.rx.rank, self.rx.world
        self._keep = None
        self.rounds = 0
        self.closing = 0  # closing exchanges (one per sharded expansion)

        def cb(user, iop):
            try:
                io = iop.contents
                cat, counts, _, t_max = self.rx.exchange(io.n_local, io.elapsed_ms, io.aux_local,
                                                         tuple(io.bbox_local), io.stream or 0)
                self._keep = cat  # the engine reads it (stream-ordered) before the next exchange
                io.dev_all = cat.data_ptr() if cat.shape[0] else None
                io.n_all = int(cat.shape[0])
                io.max_elapsed_ms = float(t_max)
                io.aux_sum = self.rx.aux_sum
                for q in range(4):
                    io.bbox_all[q] = self.rx.bbox_all[q]
                self.rounds += 1
                self.closing += bool(io.flags & 1)
                return 0
            except Exception:  # reported to the engine, which returns CLRRT_EHIP
                traceback.print_exc()
                return -1

        self._cb = EXCHANGE_FN(cb)
        planner.set_shards(self.rank, self.world, self.rx.records_ptr(), self.rx.cap, self._cb)

    @property
    def second_gathers(self):
        return self.rx.second_gathers

    @property
    def collectives(self):
        """All-gathers issued (one per round unless a round's count passed the bound)."""
        return self.rx.collectives


def exchange_capacity(max_batch, defer_steps=0, sim_dt=0.04):
    """Records one rank may commit in a round: 2 per sample of its slice and of its deferred samples (at
    most the ring's R - 1 earlier rounds: R = ceil(2 n_steps / T) + 2, clrrt_capi.hip ensure_defer)."""
    import math
    n_steps = 0
    while n_steps < 20.0 / sim_dt:
        n_steps += 1
    R = (2 * n_steps + defer_steps - 1) // defer_steps + 2 if defer_steps > 0 else 1
    return 2 * max_batch * R


def goal_sum(records):
    """Appended nodes with goalReached set (feasible paths) among the records, as a device tensor (no
    host sync: accumulate per query, read once)."""
    if records.shape[0] == 0:
        return torch.zeros((), dtype=torch.int64, device=records.device)
    return records[:, GOAL_OFFSET:GOAL_OFFSET + 4].contiguous().view(torch.int32).sum(dtype=torch.int64)


def goal_count(records):
    return int(goal_sum(records).item())


def shard(n_total, world, rank):
    """Contiguous slice [first, first + count) of a round's samples handled by `rank` (the engine's
    shard_slice, clrrt_capi.hip)."""
    first = n_total * rank // world
    return first, n_total * (rank + 1) // world - first


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
