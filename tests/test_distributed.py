"""Multi-rank frame assembly on CPU (gloo), world_size 2 and 3.

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
        assert len(fa.rows) == rtamd.shard_rows(H, row_block, rank, world_size)
        part, _ = pyoracle.OracleWorld.from_world(w).render_rows(cam.desc_bytes(), depth, fa.rows, 2)
        fa.shard[: len(fa.rows)] = torch.from_numpy(part)
        canvas = fa.assemble()
        if rank == 0:
            np.save(out_path, canvas.numpy())
        else:
            assert canvas is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world_size,row_block", [(2, 8), (3, 5), (2, 64)])
def test_gloo_frame_assembly(tmp_path, world_size, row_block):
    out = str(tmp_path / "canvas.npy")
    mp.spawn(_worker, args=(world_size, _free_port(), row_block, out), nprocs=world_size, join=True)
    got = np.load(out)
    ref = np.load(os.path.join(HERE, "golden", "c3_64x36_s200.npz"))["canvas"]
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)


def test_shard_rows_partition(rt):
    from rtamd.distributed import shard_row_ids
    for H, B, n in [(1080, 8, 8), (1080, 8, 3), (37, 5, 4), (4, 8, 8), (1, 1, 2)]:
        rows = [shard_row_ids(H, B, s, n) for s in range(n)]
        assert sorted(sum(rows, [])) == list(range(H))
        assert [len(r) for r in rows] == [rt.shard_rows(H, B, s, n) for s in range(n)]
