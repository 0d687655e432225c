"""Multi-rank path on CPU: world sizes 2 and 4 with the gloo backend, and the drop-in's 8-shard plan.

Each rank plans the reference schedule with the product's host-only context (fmgi_plan: the same
launches, rng offsets and work items on every rank), takes its shard (fmgi.parallel.shard_range) and
bakes it -- with the oracle standing in for the GPU, since this container has none -- and the int64
lightmaps are summed with fmgi.parallel.reduce_lightmap (the same call bench.py makes over RCCL). The
reduced lightmap must equal the single-process bake bit for bit, and fmgi.parallel.gather_rows (bench.py's
per-rank breakdown at N > 1) must hand every rank all ranks' rows in rank order. The drop-in's own one-process layout for
8 GPUs (fmgi_dropin_shards, fmgi_dropin_reduce_order: the peer-copy tree used without RCCL) is replayed
on per-shard lightmaps the same way."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, ORACLE, PKG


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, items, out_path):
    import sys

    sys.path[:0] = [PKG, ORACLE]
    import fm_oracle as O
    from fmgi import parallel, scene

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import fmgi

    sc = scene.box_scene(200)
    offs = np.load(os.path.join(GOLDEN, "glibc_rand_4096.npy"))
    ctx = fmgi.Context(fmgi.HOST_ONLY)  # the product's planning, as bench.py does on every rank
    ctx.set_scene(sc)
    total = ctx.plan(172_413_793, rng_offsets=offs)
    L = ctx.get_plan()
    assert L.tobytes() == O.schedule_with_offsets(sc, 172_413_793, offs).tobytes()
    assert items <= total
    b, e = parallel.shard_range(items, rank, world)
    lm3, _ = O.bake(sc, L, b, e, nthreads=2)
    lm = torch.zeros((sc.num_texels, 4), dtype=torch.int64)
    lm[:, :3] = torch.from_numpy(lm3)
    parallel.reduce_lightmap(lm, dst=0)
    # bench.py's per-rank breakdown: every rank's row, in rank order, on every rank (exact in float64)
    rows = parallel.gather_rows([rank, b, e, 100 * (e - b) + 0.5])
    assert rows == [[float(r), *map(float, parallel.shard_range(items, r, world)),
                     100.0 * (parallel.shard_range(items, r, world)[1] - parallel.shard_range(items, r, world)[0]) + 0.5]
                    for r in range(world)], rows
    if rank == 0:
        np.save(out_path, lm.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_bake_reduces_to_single_process_result(world, tmp_path, box200):
    import fm_oracle as O

    items = 300
    out = str(tmp_path / "lm.npy")
    mp.spawn(_worker, args=(world, _free_port(), items, out), nprocs=world, join=True)
    got = np.load(out)
    offs = np.load(os.path.join(GOLDEN, "glibc_rand_4096.npy"))
    L = O.schedule_with_offsets(box200, 172_413_793, offs)
    exp, _ = O.bake(box200, L, 0, items)
    assert np.array_equal(got[:, :3], exp)
    assert not got[:, 3].any()


def test_shard_ranges_tile_the_item_list():
    from fmgi import parallel

    for total in (0, 1, 7, 10_000_026, 100_000_256):
        for world in (1, 2, 3, 4, 8):
            rs = [parallel.shard_range(total, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            sizes = [e - b for b, e in rs]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        parallel.shard_range(10, 2, 2)


def test_dropin_eight_shard_plan_reduces_exactly(box200):
    """fmgi_dropin_shards for 8 GPUs: contiguous, equal item ranges on devices 0..7; summing per-shard
    lightmaps along fmgi_dropin_reduce_order (binary tree into shard 0) gives the whole bake exactly."""
    import fm_oracle as O
    import fmgi

    offs = np.load(os.path.join(GOLDEN, "glibc_rand_4096.npy"))
    ctx = fmgi.Context(fmgi.HOST_ONLY)
    ctx.set_scene(box200)
    ctx.plan(172_413_793, rng_offsets=offs)
    L = ctx.get_plan()
    items = 400
    dev, b, e = fmgi.dropin_shards(items, 8, 8)
    assert list(dev) == list(range(8)) and b[0] == 0 and e[-1] == items
    assert all(e[k] == b[k + 1] for k in range(7)) and max(e - b) - min(e - b) <= 1
    lms = [O.bake(box200, L, int(b[k]), int(e[k]), nthreads=2)[0] for k in range(8)]
    dst, src = fmgi.dropin_reduce_order(8)
    assert len(dst) == 7 and sorted(set(src)) == list(range(1, 8))
    for d, s_ in zip(dst, src):
        lms[d] = lms[d] + lms[s_]
    exp, _ = O.bake(box200, L, 0, items)
    assert np.array_equal(lms[0], exp)
