"""Multi-GPU frame assembly: one process per GPU, interleaved row blocks.

With `pattern` (block_patterns) the blocks are dealt in periods in which rank 0,
which also receives and un-interleaves every frame, owns fewer blocks than the
others (rt_render_block_pattern_device renders such a pattern).

The reference parallelises `render_multithreaded` over contiguous row blocks
of a shared canvas (camera.rs:157-172). Here the frame is split into blocks of
`row_block` rows dealt round-robin to the shards (block b -> shard b mod N, same
rule as `rt_shard_rows` / `rt_render_shard_device`, include/rt_render.h; rank r
renders shard N-1-r, `shard_of`), so
dense and empty regions spread evenly. Each rank renders its rows into a
device buffer padded to the largest shard; ONE gather (RCCL on GPUs, gloo in
the CPU tests) brings the shards to rank 0, into one contiguous buffer, which
rank 0 un-interleaves into the row-major canvas with one index_select. No other exchange exists.
"""
import torch
import torch.distributed as dist


def shard_of(rank, n_shards):
    """The shard rank `rank` renders: ranks take the shards in reverse, so
    that rank 0, which also receives and assembles every frame, renders the
    last shard, the one with the fewest rows when the row blocks do not divide
    evenly (C3 at 8 GPUs: 135 blocks, 16 for rank 0 and 17 for the others)."""
    return n_shards - 1 - rank


def shard_row_ids(height, row_block, shard, n_shards):
    """Canvas rows owned by `shard`, in the order the shard buffer stores them."""
    return [y for y in range(height) if (y // row_block) % n_shards == shard]


def pattern_row_ids(height, row_block, period, mask):
    """Canvas rows owned by a block pattern (rt_render_block_pattern_device:
    block b belongs to it iff bit b % period of mask is set), in the order its
    buffer stores them. shard_row_ids(h, b, s, n) == pattern_row_ids(h, b, n, 1 << s)."""
    return [y for y in range(height) if (mask >> ((y // row_block) % period)) & 1]


def block_patterns(n_ranks, root_share=1.0, max_period=64):
    """Row-block patterns for `n_ranks` ranks (ABI 6, rt_render_block_pattern_device):
    returns (period, masks), masks[r] the blocks of rank r. Rank 0 also receives
    and un-interleaves every frame, so it takes `root_share` of an equal share
    (rounded to what a period of at most `max_period` blocks can express); the
    others take equal shares. Within a period each rank's blocks are spread
    evenly (the position goes to the rank furthest behind its quota), so dense
    and empty regions of the frame spread over the ranks as with the plain
    interleave, which is the case root_share = 1 (period n, masks 1 << r)."""
    if n_ranks <= 1:
        return 1, [1]
    best = None
    for c in range(1, max_period + 1):
        c0 = max(1, int(round(c * root_share)))
        period = c0 + (n_ranks - 1) * c
        if period > max_period:
            break
        err = abs(c0 / c - root_share)
        if best is None or err < best[0] - 1e-9:
            best = (err, c0, c, period)
    _, c0, c, period = best
    quota = [c0] + [c] * (n_ranks - 1)
    got = [0] * n_ranks
    masks = [0] * n_ranks
    for pos in range(period):
        r = min((r for r in range(n_ranks) if got[r] < quota[r]), key=lambda r: ((got[r] + 0.5) / quota[r], r))
        masks[r] |= 1 << pos
        got[r] += 1
    return period, masks


def root_share_default(config, n_ranks):
    """Rank 0's share of an equal row split in bench.py's N-rank runs: its render
    time plus its assembly (the receive of N-1 shards and the un-interleave)
    should equal the other ranks' render time. Measured on one MI355X for C3
    (profiles/r05_assembly_n8.txt): a row block of an N-way shard renders in
    about 0.0060-0.0067 ms per frame, the un-interleave costs 0.020 ms per frame
    and the receive of 7 shards 0.014-0.015 ms, which gives about 0.97 / 0.9 /
    0.7 of an equal share at N = 2 / 4 / 8; at N = 8, 0.68 (2 of every 23 blocks
    against 3) balanced rank 0 (0.109 ms per frame with its emulated receive and
    un-interleave) with the busiest other rank (0.109 ms), where 0.75 left rank
    0 at 0.123 ms. C5 frames are 57x longer, so its assembly is within a few
    per cent of a rank's work: an equal split."""
    if config != "c3" or n_ranks <= 1:
        return 1.0
    return {2: 0.97, 4: 0.9, 8: 0.68}.get(n_ranks, max(0.6, 1.0 - 0.04 * n_ranks))


def rank_row_ids(height, row_block, rank, n_ranks, pattern=None):
    """Canvas rows rank `rank` renders: its interleaved shard (shard_of), or with
    `pattern` = block_patterns(...) its block pattern, in buffer order."""
    if pattern is None:
        return shard_row_ids(height, row_block, shard_of(rank, n_ranks), n_ranks)
    period, masks = pattern
    return pattern_row_ids(height, row_block, period, masks[rank])


class FrameAssembler:
    """Shard buffers + the gather/un-interleave step of one (H, W) frame.

    `slots` > 1 pipelines consecutive frames: frame s renders into shard slot
    s % slots, `submit(s)` issues its gather asynchronously and only then
    completes frame s-1 (wait + un-interleave), so the gather of one frame
    runs (on RCCL's stream) while the next frame renders. Stream order keeps
    it safe: a slot's shard is rendered again only after the stream has
    waited on that slot's previous gather, and a slot's gather list is
    overwritten only by a gather issued after the un-interleave that read it.
    """

    def __init__(self, height, width, row_block, rank, n_shards, device, dtype=torch.float64, slots=1, pattern=None):
        self.H, self.W, self.B = height, width, row_block
        self.rank, self.n = rank, n_shards
        self.shard_index = shard_of(rank, n_shards)
        self.pattern = pattern
        self.rows = rank_row_ids(height, row_block, rank, n_shards, pattern)
        self.max_rows = max(len(rank_row_ids(height, row_block, r, n_shards, pattern)) for r in range(n_shards))
        # padded so that every rank sends the same element count
        self.shards = [torch.zeros((self.max_rows, width, 3), dtype=dtype, device=device) for _ in range(slots)]
        self.shard = self.shards[0]
        self._pending = None  # (work, slot) of the last submitted, not yet completed frame
        if rank == 0:
            # each slot's gather lands in ONE contiguous (n * max_rows, W, 3) buffer (the
            # list handed to the gather is views of it), and the un-interleave is a single
            # index_select through the inverse row map: canvas row y <- buffer row src[y]
            self.gather_buf = [torch.empty((n_shards * self.max_rows, width, 3), dtype=dtype, device=device)
                               for _ in range(slots)]
            self.gathered = [[b[s * self.max_rows:(s + 1) * self.max_rows] for s in range(n_shards)]
                             for b in self.gather_buf]
            self.canvas = torch.empty((height, width, 3), dtype=dtype, device=device)
            inv = [0] * height
            for s in range(n_shards):  # gather position s holds rank s's shard
                for i, y in enumerate(rank_row_ids(height, row_block, s, n_shards, pattern)):
                    inv[y] = s * self.max_rows + i
            self.inv_idx = torch.tensor(inv, device=device)

    def slot(self, step):
        """Shard buffer frame `step` renders into."""
        return self.shards[step % len(self.shards)]

    def _gather(self, slot, group, async_op):
        return dist.gather(self.shards[slot], self.gathered[slot] if self.rank == 0 else None, dst=0,
                           group=group, async_op=async_op)

    def _unweave(self, slot):
        torch.index_select(self.gather_buf[slot], 0, self.inv_idx, out=self.canvas)
        return self.canvas

    def assemble(self, group=None):
        """Gather all shards to rank 0; returns the (H, W, 3) canvas on rank 0,
        None elsewhere. With one shard the shard buffer already is the canvas."""
        if self.n == 1:
            return self.shard[: self.H]
        self._gather(0, group, False)
        if self.rank != 0:
            return None
        return self._unweave(0)

    def submit(self, step, group=None):
        """Issue frame `step`'s gather, then complete frame step-1. Returns
        frame step-1's canvas on rank 0 (None elsewhere or if there is none),
        valid until the next submit."""
        if self.n == 1:
            prev, self._pending = self._pending, (None, step % len(self.shards))
            return None if prev is None else self.shards[prev[1]][: self.H]
        work = self._gather(step % len(self.shards), group, True)
        done = self._complete()
        self._pending = (work, step % len(self.shards))
        return done

    def flush(self):
        """Complete the last submitted frame; its canvas on rank 0."""
        if self.n == 1:
            prev, self._pending = self._pending, None
            return None if prev is None else self.shards[prev[1]][: self.H]
        done = self._complete()
        self._pending = None
        return done

    def _complete(self):
        if self._pending is None:
            return None
        work, slot = self._pending
        work.wait()  # NCCL: the current stream waits on the gather (the host does not block)
        return self._unweave(slot) if self.rank == 0 else None


class StreamFrameAssembler:
    """Frame assembly with frames in flight and no cross-stream coupling.

    Frames render on F streams in batches of `batch` frames (one
    rt_render_frames_device call; batch 1 = one frame per call): frame s is
    frame s % batch of batch s // batch, on stream (s // batch) % F. Each
    stream owns the shard slots of one batch (contiguous), a gather buffer and
    (on rank 0) a canvas per frame of the batch, and a process group of its
    own, so a batch's render, its ONE gather (RCCL on that group's stream,
    fenced against the render stream both ways) and rank 0's un-interleave all
    run in order behind that one stream. Batches on different streams never
    wait on each other, and slot reuse (batch + F) is ordered by the stream
    itself. The un-interleave is one index_select through the inverse row map
    (as in FrameAssembler). `streams=None` runs on the current stream (CPU
    tests with gloo).
    """

    def __init__(self, height, width, row_block, rank, n_shards, device, streams=None, groups=None,
                 dtype=torch.float64, slots=1, batch=1, pattern=None):
        self.H, self.W, self.B = height, width, row_block
        self.rank, self.n = rank, n_shards
        self.streams = streams
        self.F = len(streams) if streams else max(1, slots)
        self.NB = max(1, batch)
        self.groups = groups if groups is not None else [None] * self.F
        self.shard_index = shard_of(rank, n_shards)
        self.pattern = pattern
        self.rows = rank_row_ids(height, row_block, rank, n_shards, pattern)
        self.max_rows = max(len(rank_row_ids(height, row_block, r, n_shards, pattern)) for r in range(n_shards))
        # stream k's batch: NB padded shard slots, back to back (one gather sends them all)
        self.shards = [torch.zeros((self.NB * self.max_rows, width, 3), dtype=dtype, device=device)
                       for _ in range(self.F)]
        self.shard = self.shards[0][: self.max_rows]
        self._last = None
        if rank == 0 and n_shards > 1:
            per = self.NB * self.max_rows  # rows rank s sends
            self.gather_buf = [torch.empty((n_shards * per, width, 3), dtype=dtype, device=device)
                               for _ in range(self.F)]
            self.gathered = [[b[s * per:(s + 1) * per] for s in range(n_shards)] for b in self.gather_buf]
            self.canvas = [torch.empty((self.NB * height, width, 3), dtype=dtype, device=device)
                           for _ in range(self.F)]
            one, inv = [0] * height, [0] * (self.NB * height)
            for s in range(n_shards):  # gather position s holds rank s's shard slots
                for i, y in enumerate(rank_row_ids(height, row_block, s, n_shards, pattern)):
                    one[y] = s * self.max_rows + i  # one frame's gather (no batch)
                    for j in range(self.NB):  # canvas j, row y <- rank s's slot j, row i
                        inv[j * height + y] = s * per + j * self.max_rows + i
            self.inv_idx = torch.tensor(one, device=device)
            self.inv_batch = torch.tensor(inv, device=device)

    def _k(self, step):
        return (step // self.NB) % self.F

    def slot(self, step):
        """Shard buffer frame `step` renders into (on stream (step // batch) % F)."""
        j = step % self.NB
        return self.shards[self._k(step)][j * self.max_rows:(j + 1) * self.max_rows]

    def stream(self, step):
        return self.streams[self._k(step)] if self.streams else None

    def submit(self, step, end=None):
        """Frame `step` is rendered. At the end of its batch (`end`, default:
        the batch's last frame) gather and assemble the batch, queued behind
        its render on its stream; returns frame step's canvas on rank 0 (valid
        until batch step // batch + F is submitted), None elsewhere or before
        the batch's end."""
        k, j = self._k(step), step % self.NB
        if self.n == 1:
            self._last = self.slot(step)[: self.H]
            return self._last
        if end is None:
            end = j == self.NB - 1
        if not end:
            return None
        ctx = torch.cuda.stream(self.streams[k]) if self.streams else _nullctx()
        with ctx:
            self._gather(k)
            if self.rank != 0:
                self._last = None
                return None
            torch.index_select(self.gather_buf[k], 0, self.inv_batch, out=self.canvas[k])
            self._last = self.canvas[k][j * self.H:(j + 1) * self.H]
            return self._last

    def _gather(self, k):
        work = dist.gather(self.shards[k], self.gathered[k] if self.rank == 0 else None, dst=0,
                           group=self.groups[k], async_op=True)
        work.wait()  # the batch's stream waits on its gather (the host does not block)

    def flush(self):
        """The last submitted frame's canvas on rank 0 (everything is already queued)."""
        return self._last


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


class RcclStreamAssembler(StreamFrameAssembler):
    """StreamFrameAssembler whose gathers are RCCL collectives the library
    enqueues directly on each frame's render stream (one communicator per
    render stream, rtamd._rtamd._nccl_*): a frame's render, gather and rank
    0's un-interleave are consecutive work of ONE stream, with no
    cross-stream event at all. Cross-stream fences (a render stream and a
    process group's own RCCL stream waiting on each other) cost ~0.17 ms per
    frame on an 8-way shard (`bench.py --fake-shard 0/8 --emulate-gather`),
    which is the whole frame again. The communicators' unique ids travel over
    the default process group.

    Creation is all-or-nothing across ranks: after each communicator every
    rank contributes its success to a MIN all-reduce over the default group
    (the library creates communicators non-blocking with a timeout, so a rank
    whose peers failed does not hang in the init). If any rank failed, every
    rank aborts what it created and raises together, so all ranks take the
    caller's fallback in step. `lib` (tests) replaces the library hooks;
    `streams` entries may be None (CPU tests: the current stream)."""

    def __init__(self, height, width, row_block, rank, n_shards, device, streams, dtype=torch.float64, lib=None,
                 timeout_ms=60000, batch=1, pattern=None):
        super().__init__(height, width, row_block, rank, n_shards, device, streams=streams,
                         groups=[None] * len(streams), dtype=dtype, batch=batch, pattern=pattern)
        if lib is None:
            from . import _rtamd as lib
        self._lib = lib
        if device.type == "cuda":
            dev_index = device.index if device.index is not None else torch.cuda.current_device()
        else:
            dev_index = 0
        self.comms = []
        try:
            for _ in range(self.F):
                # byte 0: rank 0 could make an id (1) or not (0); every rank reads the same flag
                msg = torch.zeros(129, dtype=torch.uint8, device=device)
                if rank == 0:
                    try:
                        msg[1:].copy_(torch.frombuffer(bytearray(lib._nccl_unique_id()), dtype=torch.uint8))
                        msg[0] = 1
                    except Exception:  # pragma: no cover - environment dependent
                        msg[0] = 0
                dist.broadcast(msg, src=0)
                host = msg.cpu().numpy().tobytes()
                if host[0] != 1:
                    raise RuntimeError("rank 0 could not create an RCCL unique id")
                comm, err = None, None
                try:
                    comm = lib._nccl_comm_init(n_shards, host[1:], rank, dev_index, timeout_ms)
                except Exception as e:
                    err = e
                if comm is not None:
                    self.comms.append(comm)
                ok = torch.tensor([1 if comm is not None else 0], dtype=torch.int32, device=device)
                dist.all_reduce(ok, op=dist.ReduceOp.MIN)
                if int(ok[0]) != 1:
                    raise RuntimeError(f"RCCL communicator creation failed on some rank"
                                       f"{f' (here: {err})' if err is not None else ''}")
        except Exception:
            self.abort()
            raise

    def _stream_handle(self, k):
        st = self.streams[k]
        return (st.cuda_stream if st is not None else 0), st

    def submit(self, step, end=None):
        k = self._k(step)
        if self.n == 1 or self.streams[k] is None:
            return super().submit(step, end)
        with torch.cuda.stream(self.streams[k]):  # index_select on the render stream, behind the gather
            return super().submit(step, end)

    def _gather(self, k):
        handle, _ = self._stream_handle(k)
        recv = self.gather_buf[k].data_ptr() if self.rank == 0 else 0
        self._lib._nccl_gather_f64(self.shards[k].data_ptr(), recv, self.shards[k].numel(), 0, self.comms[k], handle)

    def abort(self):
        """Tear the communicators down without waiting on peers (failure path)."""
        for c in self.comms:
            try:
                self._lib._nccl_comm_abort(c)
            except Exception:  # pragma: no cover - best effort
                pass
        self.comms = []

    def close(self):
        for c in self.comms:
            self._lib._nccl_comm_destroy(c)
        self.comms = []
