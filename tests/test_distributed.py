"""Multi-rank frame assembly on CPU (gloo), world_size 2, 3 and 8.

Each rank renders ONLY its interleaved row blocks (rtamd.distributed, the same
layout as rt_render_shard_device) — here with the oracle, since this container
has no GPU — into the padded shard buffer; FrameAssembler gathers them to rank
0 and un-interleaves. The assembled canvas must equal the golden full frame
bit for bit (N-GPU output bit-identical to 1 GPU).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world_size, port, row_block, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        import rtamd
        from rtamd.distributed import FrameAssembler
        from oracle import pyoracle
        import golden_cases
        w, cam, depth = golden_cases.scene(rtamd, "c3", {"width": 64, "height": 36, "n_spheres": 200})
        H, W = cam.vsize, cam.hsize
        fa = FrameAssembler(H, W, row_block, rank, world_size, torch.device("cpu"))
        assert len(fa.rows) == rtamd.shard_rows(H, row_block, world_size - 1 - rank, world_size)
        part, _ = pyoracle.OracleWorld.from_world(w).render_rows(cam.desc_bytes(), depth, fa.rows, 2)
        fa.shard[: len(fa.rows)] = torch.from_numpy(part)
        canvas = fa.assemble()
        if rank == 0:
            np.save(out_path, canvas.numpy())
        else:
            assert canvas is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world_size,row_block", [(2, 8), (3, 5), (2, 64), (8, 4)])
def test_gloo_frame_assembly(tmp_path, world_size, row_block):
    out = str(tmp_path / "canvas.npy")
    mp.spawn(_worker, args=(world_size, _free_port(), row_block, out), nprocs=world_size, join=True)
    got = np.load(out)
    ref = np.load(os.path.join(HERE, "golden", "c3_64x36_s200.npz"))["canvas"]
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)


def _pipeline_worker(rank, world_size, port, row_block, n_frames, out_path):
    """Frame f is golden + f; frames go through the 2-slot pipeline."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from rtamd.distributed import FrameAssembler
        ref = torch.from_numpy(np.load(os.path.join(HERE, "golden", "c3_64x36_s200.npz"))["canvas"])
        H, W = ref.shape[:2]
        fa = FrameAssembler(H, W, row_block, rank, world_size, torch.device("cpu"), slots=2)
        done = []
        for f in range(n_frames):
            buf = fa.slot(f)
            buf.fill_(-1.0)
            buf[: len(fa.rows)] = ref[fa.rows] + f
            c = fa.submit(f)
            if f == 0 or rank != 0:
                assert c is None
            else:
                done.append(c.clone())
        c = fa.flush()
        if rank == 0:
            done.append(c.clone())
            np.save(out_path, torch.stack(done).numpy())
        else:
            assert c is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world_size,row_block", [(2, 8), (3, 5)])
def test_gloo_pipelined_frames(tmp_path, world_size, row_block):
    """The 2-slot pipeline bench.py runs at N>1: every frame comes out whole
    and in order, one submit behind."""
    out = str(tmp_path / "frames.npy")
    mp.spawn(_pipeline_worker, args=(world_size, _free_port(), row_block, 5, out), nprocs=world_size, join=True)
    got = np.load(out)
    ref = np.load(os.path.join(HERE, "golden", "c3_64x36_s200.npz"))["canvas"]
    assert got.shape == (5,) + ref.shape
    for f in range(5):
        assert np.array_equal(got[f], ref + f), f


def test_single_shard_pipeline():
    from rtamd.distributed import FrameAssembler
    fa = FrameAssembler(10, 4, 8, 0, 1, torch.device("cpu"), slots=2)
    outs = []
    for f in range(3):
        fa.slot(f).fill_(f)
        c = fa.submit(f)
        outs.append(None if c is None else float(c[0, 0, 0]))
    outs.append(float(fa.flush()[9, 3, 2]))
    assert outs == [None, 0.0, 1.0, 2.0]


def test_shard_rows_partition(rt):
    from rtamd.distributed import shard_row_ids
    for H, B, n in [(1080, 8, 8), (1080, 8, 3), (37, 5, 4), (4, 8, 8), (1, 1, 2)]:
        rows = [shard_row_ids(H, B, s, n) for s in range(n)]
        assert sorted(sum(rows, [])) == list(range(H))
        assert [len(r) for r in rows] == [rt.shard_rows(H, B, s, n) for s in range(n)]


def _batch_done(fa, f, batch, n_frames, c, done):
    """Rank 0's canvases of the batch that frame f ends (if it ends one)."""
    if f % batch != batch - 1 and f != n_frames - 1:
        assert c is None
        return
    k = (f // batch) % fa.F
    for g in range(f - f % batch, f + 1):
        done.append(fa.canvas[k][(g % batch) * fa.H:(g % batch + 1) * fa.H].clone())
    assert torch.equal(c, done[-1])


def _ref_canvas(kind):
    """The frame every test frame is derived from: the golden C3 64x36 frame, or
    ("c3rows") a synthetic canvas of C3's full height, 1080 rows (135 blocks of 8
    at 8 ranks: 16 for rank 0, 17 for the others, as bench.py's N=8 run), with
    every row and column distinct."""
    if kind == "golden":
        return torch.from_numpy(np.load(os.path.join(HERE, "golden", "c3_64x36_s200.npz"))["canvas"])
    H, W = (4096, 4) if kind == "c5rows" else (1080, 6)  # C5: 4096 rows, 512 blocks of 8
    y = torch.arange(H, dtype=torch.float64).view(H, 1, 1)
    x = torch.arange(W, dtype=torch.float64).view(1, W, 1)
    c = torch.arange(3, dtype=torch.float64).view(1, 1, 3)
    return y * 1000.0 + x * 10.0 + c / 4.0


def _stream_worker(rank, world_size, port, row_block, n_frames, n_slots, out_path, batch=1, kind="golden",
                   share=None):
    """StreamFrameAssembler (bench.py's N>1 path): frame f is golden + f, one
    process group per slot; every submit returns frame f assembled (batch > 1:
    every batch's last submit gathers and assembles the batch). `share`: rank
    0's share of the rows (block patterns, bench.py --root-share)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from rtamd.distributed import StreamFrameAssembler, block_patterns
        ref = _ref_canvas(kind)
        H, W = ref.shape[:2]
        groups = [dist.new_group(list(range(world_size))) for _ in range(n_slots)]
        pattern = block_patterns(world_size, share) if share is not None else None
        fa = StreamFrameAssembler(H, W, row_block, rank, world_size, torch.device("cpu"), groups=groups,
                                  slots=n_slots, batch=batch, pattern=pattern)
        if pattern is not None:
            import rtamd
            assert len(fa.rows) == rtamd.pattern_rows(H, row_block, pattern[0], pattern[1][rank])
        done = []
        for f in range(n_frames):
            buf = fa.slot(f)
            buf.fill_(-1.0)
            buf[: len(fa.rows)] = ref[fa.rows] + f
            if batch > 1:
                c = fa.submit(f, end=f % batch == batch - 1 or f == n_frames - 1)
                if rank == 0:
                    _batch_done(fa, f, batch, n_frames, c, done)
                else:
                    assert c is None
                continue
            c = fa.submit(f)
            if rank == 0:
                done.append(c.clone())
            else:
                assert c is None
        if rank == 0:
            assert fa.flush() is not None
            np.save(out_path, torch.stack(done).numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world_size,row_block,n_slots", [(2, 8, 4), (3, 5, 3)])
def test_gloo_stream_assembler(tmp_path, world_size, row_block, n_slots):
    """The per-stream assembler of bench.py's N>1 path (one slot, gather buffer,
    canvas and process group per render stream): every frame comes out whole."""
    out = str(tmp_path / "frames.npy")
    mp.spawn(_stream_worker, args=(world_size, _free_port(), row_block, 6, n_slots, out), nprocs=world_size,
             join=True)
    got = np.load(out)
    ref = np.load(os.path.join(HERE, "golden", "c3_64x36_s200.npz"))["canvas"]
    assert got.shape == (6,) + ref.shape
    for f in range(6):
        assert np.array_equal(got[f], ref + f), f


@pytest.mark.parametrize("world_size,row_block,n_slots,batch", [(2, 8, 2, 4), (3, 5, 3, 3)])
def test_gloo_stream_assembler_batches(tmp_path, world_size, row_block, n_slots, batch):
    """Batches of frames (bench.py --batch: one render call and ONE gather per
    batch): 11 frames, the last batch partial, every frame comes out whole."""
    out = str(tmp_path / "frames.npy")
    mp.spawn(_stream_worker, args=(world_size, _free_port(), row_block, 11, n_slots, out, batch), nprocs=world_size,
             join=True)
    got = np.load(out)
    ref = np.load(os.path.join(HERE, "golden", "c3_64x36_s200.npz"))["canvas"]
    assert got.shape == (11,) + ref.shape
    for f in range(11):
        assert np.array_equal(got[f], ref + f), f


class _FakeRccl:
    """Stands in for the library's RCCL hooks (rtamd._rtamd._nccl_*) on CPU:
    ids are bytes, communicators are integers, the gather runs over gloo on the
    tensors the pointers name. `fail_at` = (rank, k): that rank's k-th
    communicator init raises, as a failing ncclCommInitRankConfig would."""

    def __init__(self, rank, fail_at=None):
        self.rank, self.fail_at = rank, fail_at
        self.made, self.aborted, self.destroyed, self.gathers = [], [], [], []
        self.tensors = {}  # data_ptr -> tensor (set by the test once the assembler exists)

    def _nccl_unique_id(self):
        return bytes(range(128))

    def _nccl_comm_init(self, nranks, uid, rank, dev, timeout_ms):
        assert uid == bytes(range(128)) and rank == self.rank and timeout_ms > 0
        k = len(self.made) + len(self.aborted)
        if self.fail_at == (rank, k):
            raise RuntimeError("injected ncclCommInitRankConfig failure")
        c = 1000 * (rank + 1) + k
        self.made.append(c)
        return c

    def _nccl_comm_abort(self, c):
        self.aborted.append(c)

    def _nccl_comm_destroy(self, c):
        self.destroyed.append(c)

    def _nccl_gather_f64(self, send, recv, count, root, comm, stream):
        self.gathers.append((send, comm, stream))
        src = self.tensors[send]
        assert src.numel() == count and root == 0
        if self.rank == 0:
            dst = self.tensors[recv]
            dist.gather(src, list(dst.chunk(dist.get_world_size())), dst=0)
        else:
            dist.gather(src, None, dst=0)


def _rccl_assembler_worker(rank, world_size, port, fail_at, n_frames, out_path, batch=1, kind="golden", F=3,
                           share=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from rtamd.distributed import RcclStreamAssembler, block_patterns
        pattern = block_patterns(world_size, share) if share is not None else None
        ref = _ref_canvas(kind)
        H, W = ref.shape[:2]
        lib = _FakeRccl(rank, fail_at)
        if fail_at is not None:
            with pytest.raises(RuntimeError, match="failed on some rank"):
                RcclStreamAssembler(H, W, 8, rank, world_size, torch.device("cpu"), streams=[None] * F, lib=lib)
            # every rank fell back together and left nothing behind
            assert sorted(lib.aborted) == sorted(lib.made) and not lib.destroyed
            assert len(lib.made) == fail_at[1] + (0 if rank == fail_at[0] else 1)
            dist.barrier()  # the default group still works: nobody is stuck in an init
            np.save(out_path + f".{rank}", np.array([len(lib.made)]))
            return
        fa = RcclStreamAssembler(H, W, 8, rank, world_size, torch.device("cpu"), streams=[None] * F, lib=lib,
                                 batch=batch, pattern=pattern)
        assert fa.comms == [1000 * (rank + 1) + k for k in range(F)]
        for t in fa.shards:
            lib.tensors[t.data_ptr()] = t
        if rank == 0:
            for t in fa.gather_buf:
                lib.tensors[t.data_ptr()] = t
        done = []
        for f in range(n_frames):
            buf = fa.slot(f)
            buf.fill_(-1.0)
            buf[: len(fa.rows)] = ref[fa.rows] + f
            if batch > 1:
                n_before = len(lib.gathers)
                end = f % batch == batch - 1 or f == n_frames - 1
                c = fa.submit(f, end=end)
                # one gather per batch, of the batch's slots, over communicator (f // batch) % F
                assert len(lib.gathers) == n_before + (1 if end else 0)
                if end:
                    k = (f // batch) % F
                    assert lib.gathers[-1][:2] == (fa.shards[k].data_ptr(), fa.comms[k])
                if rank == 0:
                    _batch_done(fa, f, batch, n_frames, c, done)
                else:
                    assert c is None
                continue
            c = fa.submit(f)
            # frame f gathers slot f % F over communicator f % F
            assert lib.gathers[-1][:2] == (fa.shards[f % F].data_ptr(), fa.comms[f % F])
            if rank == 0:
                done.append(c.clone())
            else:
                assert c is None
        fa.close()
        assert lib.destroyed == [1000 * (rank + 1) + k for k in range(F)] and not lib.aborted
        if rank == 0:
            np.save(out_path, torch.stack(done).numpy())
    finally:
        dist.destroy_process_group()


def test_gloo_rccl_stream_assembler_frames(tmp_path):
    """bench.py's default N>1 assembler (one library communicator per render
    stream): id broadcast, per-slot communicators, frame f through slot and
    communicator f % F, every frame assembled whole."""
    out = str(tmp_path / "frames.npy")
    mp.spawn(_rccl_assembler_worker, args=(2, _free_port(), None, 7, out), nprocs=2, join=True)
    got = np.load(out)
    ref = np.load(os.path.join(HERE, "golden", "c3_64x36_s200.npz"))["canvas"]
    for f in range(7):
        assert np.array_equal(got[f], ref + f), f


def test_gloo_rccl_stream_assembler_batches(tmp_path):
    """The RCCL assembler with batches: one library gather per batch."""
    out = str(tmp_path / "frames.npy")
    mp.spawn(_rccl_assembler_worker, args=(2, _free_port(), None, 13, out, 4), nprocs=2, join=True)
    got = np.load(out)
    ref = np.load(os.path.join(HERE, "golden", "c3_64x36_s200.npz"))["canvas"]
    assert got.shape == (13,) + ref.shape
    for f in range(13):
        assert np.array_equal(got[f], ref + f), f


@pytest.mark.parametrize("fail_at", [(1, 1), (0, 0), (1, 2)])
def test_gloo_rccl_stream_assembler_fallback_agreement(tmp_path, fail_at):
    """One rank's communicator init fails: every rank raises together (no rank
    left blocked in an init or a collective) and aborts what it created."""
    out = str(tmp_path / "made.npy")
    mp.spawn(_rccl_assembler_worker, args=(2, _free_port(), fail_at, 0, out), nprocs=2, join=True)
    for r in range(2):
        made = int(np.load(out + f".{r}.npy")[0])
        assert made == fail_at[1] + (0 if r == fail_at[0] else 1)


# bench.py's N = 8 run (SCALE at 8 GPUs): batches of 16 frames on 4 render
# streams (bench.py: NB = 16 for n >= 4, F = 4), 8-row blocks of C3's 1080 rows,
# K = 64 timed frames after the setup batches; here 69 frames, so the last batch
# is partial (5 frames) and the slots wrap around the 4 streams more than once.
@pytest.mark.parametrize("world_size", [4, 8])
def test_gloo_stream_assembler_bench_n8_config(tmp_path, world_size):
    out = str(tmp_path / "frames.npy")
    n_frames = 69
    mp.spawn(_stream_worker, args=(world_size, _free_port(), 8, n_frames, 4, out, 16, "c3rows"),
             nprocs=world_size, join=True)
    got = np.load(out)
    ref = _ref_canvas("c3rows").numpy()
    assert got.shape == (n_frames,) + ref.shape
    for f in range(n_frames):
        assert np.array_equal(got[f], ref + f), f


@pytest.mark.parametrize("world_size", [4, 8])
def test_gloo_rccl_stream_assembler_bench_n8_config(tmp_path, world_size):
    """The default N>1 assembler (library communicators, faked) in the same
    configuration: one gather per batch of 16 over communicator (batch mod 4)."""
    out = str(tmp_path / "frames.npy")
    n_frames = 69
    mp.spawn(_rccl_assembler_worker, args=(world_size, _free_port(), None, n_frames, out, 16, "c3rows", 4),
             nprocs=world_size, join=True)
    got = np.load(out)
    ref = _ref_canvas("c3rows").numpy()
    assert got.shape == (n_frames,) + ref.shape
    for f in range(n_frames):
        assert np.array_equal(got[f], ref + f), f


# bench.py's C5 run at 8 GPUs (--config c5): batches of one frame, ONE render
# stream (bench.py: F = 1, NB = 1 for C5), so StreamFrameAssembler gathers on
# the current stream over one process group; 4096 rows in 8-row blocks (512
# blocks, 64 per rank). Every assembled frame whole and in order.
def test_gloo_stream_assembler_bench_c5_n8_config(tmp_path):
    out = str(tmp_path / "frames.npy")
    n_frames = 5
    mp.spawn(_stream_worker, args=(8, _free_port(), 8, n_frames, 1, out, 1, "c5rows"), nprocs=8, join=True)
    got = np.load(out)
    ref = _ref_canvas("c5rows").numpy()
    assert got.shape == (n_frames,) + ref.shape
    for f in range(n_frames):
        assert np.array_equal(got[f], ref + f), f


# The N = 4 / 8 runs' uneven split (bench.py: root_share_default for C3): rank 0,
# which assembles every frame, renders fewer row blocks (block patterns, ABI 6).
@pytest.mark.parametrize("world_size,share", [(8, 0.68), (4, 0.9), (2, 0.97)])
def test_gloo_stream_assembler_root_share(tmp_path, world_size, share):
    out = str(tmp_path / "frames.npy")
    n_frames = 37
    mp.spawn(_stream_worker, args=(world_size, _free_port(), 8, n_frames, 4, out, 16, "c3rows", share),
             nprocs=world_size, join=True)
    got = np.load(out)
    ref = _ref_canvas("c3rows").numpy()
    assert got.shape == (n_frames,) + ref.shape
    for f in range(n_frames):
        assert np.array_equal(got[f], ref + f), f


@pytest.mark.parametrize("world_size", [8])
def test_gloo_rccl_stream_assembler_root_share(tmp_path, world_size):
    """The default N>1 assembler (library communicators, faked) with bench.py's
    N = 8 split of C3 (rank 0 at 0.68 of an equal share)."""
    out = str(tmp_path / "frames.npy")
    n_frames = 37
    mp.spawn(_rccl_assembler_worker, args=(world_size, _free_port(), None, n_frames, out, 16, "c3rows", 4, 0.68),
             nprocs=world_size, join=True)
    got = np.load(out)
    ref = _ref_canvas("c3rows").numpy()
    for f in range(n_frames):
        assert np.array_equal(got[f], ref + f), f
