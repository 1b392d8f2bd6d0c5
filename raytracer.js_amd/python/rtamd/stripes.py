"""Row-stripe partition of a frame across ranks, and its reassembly on rank 0.

The reference renders a frame on one CPU thread (src/raytracer.ts:309-330, Raytracer.trace_frame).
Pixels are independent, so the multi-GPU path splits the frame into stripes of `stripe` rows dealt
round-robin to ranks (rank p owns stripes p, p+N, p+2N, ...: every rank gets a share of the
expensive and the cheap parts of the image).  Each rank traces its rows into a dense local buffer
(rt_trace_rows_device, rows in stripe order) and one collective gather moves the buffers to rank 0,
which de-interleaves them into frame order with one index_select.  No other exchange exists on the
data path.

`StripeGather` holds the buffers and the row index; it works with any torch.distributed backend
(RCCL on the GPU box, gloo for the CPU tests) and with world_size 1 (the local buffer is the frame).
"""
import numpy as np
import torch
import torch.distributed as dist


def part_rows(H, part, n_parts, stripe):
    """Global row indices owned by `part`, in the order rt_trace_rows_device writes them
    (mirrors rt_part_rows in csrc/rt_internal.h)."""
    if n_parts < 1 or not (0 <= part < n_parts) or stripe < 1:
        raise ValueError("bad partition part=%r n_parts=%r stripe=%r" % (part, n_parts, stripe))
    rows = []
    n_stripes = (H + stripe - 1) // stripe
    for s in range(part, n_stripes, n_parts):
        rows.extend(range(s * stripe, min(H, (s + 1) * stripe)))
    return np.array(rows, dtype=np.int64)


def source_index(H, n_parts, stripe):
    """For every frame row y: its row in the stacked [n_parts * max_rows] gather buffer."""
    max_rows = max(len(part_rows(H, p, n_parts, stripe)) for p in range(n_parts))
    src = np.full(H, -1, np.int64)
    for p in range(n_parts):
        gr = part_rows(H, p, n_parts, stripe)
        src[gr] = p * max_rows + np.arange(len(gr))
    assert (src >= 0).all(), "partition does not cover the frame"
    return src, max_rows


class StripeGather:
    """Local stripe buffer of this rank + reassembly of the frame on rank 0.

    local   [max_rows, W, C] tensor the rank's rows are traced into (rows beyond the rank's own
            count are padding so every rank contributes an equal-sized buffer to the gather)
    frame   [H, W, C] tensor on rank 0 after gather(); None elsewhere
    """

    def __init__(self, H, W, rank, world, stripe, device, channels=3, dtype=torch.float32):
        self.H, self.W, self.rank, self.world, self.stripe = H, W, rank, world, stripe
        src, self.max_rows = source_index(H, world, stripe)
        self.rows = len(part_rows(H, rank, world, stripe))
        self.local = torch.zeros((self.max_rows, W, channels), dtype=dtype, device=device)
        if world == 1:
            self.frame = self.local          # one part: rows are already in frame order, nothing to move
        else:
            self.frame = torch.zeros((H, W, channels), dtype=dtype, device=device) if rank == 0 else None
        if world > 1 and rank == 0:
            # the ranks' buffers land in one stacked tensor (views), de-interleaved without a restack
            self._stack = torch.empty((world,) + tuple(self.local.shape), dtype=dtype, device=device)
            self._bufs = list(self._stack.unbind(0))
            self._src = torch.from_numpy(src).to(device)
        else:
            self._stack, self._bufs, self._src = None, None, None
        if self.local.is_cuda:
            # the fills ran on torch's stream; rt_trace_rows_device writes `local` on another one
            torch.cuda.synchronize(self.local.device)

    def gather(self):
        """Collective (every rank calls it): rank 0's `frame` receives the whole image."""
        if self.world == 1:
            return self.frame
        dist.gather(self.local, self._bufs if self.rank == 0 else None, dst=0)
        if self.rank == 0:
            flat = self._stack.view(self.world * self.max_rows, self.W, -1)
            torch.index_select(flat, 0, self._src, out=self.frame)
            return self.frame
        return None
