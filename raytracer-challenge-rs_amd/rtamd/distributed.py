"""Multi-GPU frame assembly: one process per GPU, interleaved row blocks.

The reference parallelises `render_multithreaded` over contiguous row blocks
of a shared canvas (camera.rs:157-172). Here the frame is split into blocks of
`row_block` rows dealt round-robin to the ranks (block b -> rank b mod N, same
rule as `rt_shard_rows` / `rt_render_shard_device`, include/rt_render.h), so
dense and empty regions spread evenly. Each rank renders its rows into a
device buffer padded to the largest shard; ONE gather (RCCL on GPUs, gloo in
the CPU tests) brings the shards to rank 0, which un-interleaves them into the
row-major canvas with one index_copy. No other exchange exists.
"""
import torch
import torch.distributed as dist


def shard_row_ids(height, row_block, shard, n_shards):
    """Canvas rows owned by `shard`, in the order the shard buffer stores them."""
    return [y for y in range(height) if (y // row_block) % n_shards == shard]


class FrameAssembler:
    """Shard buffers + the gather/un-interleave step of one (H, W) frame."""

    def __init__(self, height, width, row_block, rank, n_shards, device, dtype=torch.float64):
        self.H, self.W, self.B = height, width, row_block
        self.rank, self.n = rank, n_shards
        self.rows = shard_row_ids(height, row_block, rank, n_shards)
        self.max_rows = max(len(shard_row_ids(height, row_block, s, n_shards)) for s in range(n_shards))
        # padded so that every rank sends the same element count
        self.shard = torch.zeros((self.max_rows, width, 3), dtype=dtype, device=device)
        if rank == 0:
            self.gathered = [torch.empty_like(self.shard) for _ in range(n_shards)]
            self.canvas = torch.empty((height, width, 3), dtype=dtype, device=device)
            src, dst = [], []
            for s in range(n_shards):
                rows_s = shard_row_ids(height, row_block, s, n_shards)
                src += [s * self.max_rows + i for i in range(len(rows_s))]
                dst += rows_s
            self.src_idx = torch.tensor(src, device=device)
            self.dst_idx = torch.tensor(dst, device=device)

    def assemble(self, group=None):
        """Gather all shards to rank 0; returns the (H, W, 3) canvas on rank 0,
        None elsewhere. With one shard the shard buffer already is the canvas."""
        if self.n == 1:
            return self.shard[: self.H]
        dist.gather(self.shard, self.gathered if self.rank == 0 else None, dst=0, group=group)
        if self.rank != 0:
            return None
        self.canvas.index_copy_(0, self.dst_idx, torch.cat(self.gathered).index_select(0, self.src_idx))
        return self.canvas
