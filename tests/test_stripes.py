"""The N>1 path: row-stripe partition, collective gather to rank 0 and de-interleave.

CPU: the partition covers every row once, and a world_size-2 gloo run of rtamd.stripes.StripeGather
(each rank renders its own rows with the oracle) reassembles exactly the oracle's full frame.
GPU: rt_trace_rows_device part by part on one device, reassembled with the same row index,
equals the single-part frame bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
import rtamd
from rtamd import scenes
from rtamd.stripes import StripeGather, part_rows, source_index


@pytest.mark.parametrize("H,n,stripe", [(1080, 1, 8), (1080, 2, 8), (1080, 8, 8), (1080, 3, 7), (17, 4, 8),
                                        (5, 8, 1), (256, 5, 16)])
def test_partition_covers_each_row_once(H, n, stripe):
    rows = [part_rows(H, p, n, stripe) for p in range(n)]
    allr = np.concatenate(rows)
    assert np.array_equal(np.sort(allr), np.arange(H))
    src, max_rows = source_index(H, n, stripe)
    assert max_rows == max(len(r) for r in rows)
    for p, r in enumerate(rows):
        assert np.array_equal(src[r], p * max_rows + np.arange(len(r)))
        assert np.all(np.diff(r) > 0)                   # stripe order == increasing rows


def test_partition_rejects_bad_arguments():
    with pytest.raises(ValueError):
        part_rows(10, 2, 2, 8)
    with pytest.raises(ValueError):
        part_rows(10, 0, 1, 0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_rows(spec, cam, cfg, rows):
    """The rows' pixels rendered by the oracle, as a [len(rows), W, 3] float32 array."""
    w, root = oracle.build_scene(spec)
    W = cam.width
    pix = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1).astype(np.int32)
    r = w.trace_frame(root, cam, cfg, pixels=pix, nthreads=1)
    w.close()
    return r["rgb"].reshape(-1, 3)[pix].reshape(len(rows), W, 3)


def _worker(rank, world, port, W, H, stripe, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        spec = scenes.config1_spheres()
        cam, cfg = scenes.make_camera(W, H), scenes.make_config(2)
        sg = StripeGather(H, W, rank, world, stripe, torch.device("cpu"))
        mine = part_rows(H, rank, world, stripe)
        assert sg.rows == len(mine)
        sg.local.fill_(float("nan"))                    # padding rows must never reach the frame
        sg.local[:len(mine)] = torch.from_numpy(_oracle_rows(spec, cam, cfg, mine))
        frame = sg.gather()
        if rank == 0:
            np.save(out_path, frame.numpy())
        else:
            assert frame is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("stripe", [8, 3])
def test_gloo_world2_gather_equals_oracle_frame(tmp_path, stripe):
    W, H = 48, 37
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(2, _free_port(), W, H, stripe, out), nprocs=2, join=True,
                       start_method="spawn")
    got = np.load(out)
    spec = scenes.config1_spheres()
    cam, cfg = scenes.make_camera(W, H), scenes.make_config(2)
    w, root = oracle.build_scene(spec)
    ref = w.trace_frame(root, cam, cfg, nthreads=4)["rgb"].reshape(H, W, 3)
    w.close()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("n,stripe", [(2, 8), (3, 8), (8, 8), (5, 1)])
def test_parts_reassemble_to_full_frame_gpu(n, stripe):
    W, H = 200, 120
    spec = scenes.config1_spheres()
    cam, cfg = scenes.make_camera(W, H), scenes.make_config(2)
    ctx = rtamd.Context(0)
    try:
        ctx.upload(rtamd.build_scene(spec))
        dev = torch.device("cuda", 0)
        s = torch.cuda.Stream(device=dev)
        full = StripeGather(H, W, 0, 1, stripe, dev)
        rows, _ = ctx.trace_rows_device(cam, cfg, 0, 1, stripe, full.local.data_ptr(), s.cuda_stream)
        assert rows == H
        src, max_rows = source_index(H, n, stripe)
        stacked = torch.full((n * max_rows, W, 3), float("nan"), dtype=torch.float32, device=dev)
        torch.cuda.synchronize()                    # the fills run on torch's stream, the frames on `s`
        for p in range(n):
            rows, _ = ctx.trace_rows_device(cam, cfg, p, n, stripe, stacked[p * max_rows].data_ptr(), s.cuda_stream)
            assert rows == len(part_rows(H, p, n, stripe))
        s.synchronize()
        got = torch.index_select(stacked, 0, torch.from_numpy(src).to(dev)).cpu().numpy()
        ref = full.local[:H].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    finally:
        ctx.close()
