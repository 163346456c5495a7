"""CPU multi-process (gloo, world_size 2/3) tests of the data-parallel path: weight broadcast
bit-equality, all-gather order, ragged shard padding, and sharded deconvnet == single process."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from deconv_api_amd.parallel import dist as pdist

    return pdist.init(backend="gloo", device_type="cpu")


def _worker_collectives(rank, world, port, q):
    try:
        from deconv_api_amd.models.vgg16 import VGG16
        from deconv_api_amd.parallel import dist as pdist

        info = _init(rank, world, port)
        m = VGG16.random(0 if rank == 0 else 99, include_top=False)
        sd = pdist.broadcast_state(m.state_dict(), info, bucket_bytes=8 << 20)
        ref = VGG16.random(0, include_top=False).state_dict()
        same = all(torch.equal(sd[k], ref[k]) for k in ref)
        x = torch.full((2, 3), float(rank))
        g = pdist.all_gather_rows(x, info)
        order = g[:, 0].tolist()
        mx = pdist.all_reduce_max(float(rank) * 1.5, info)
        q.put((rank, same, order, mx))
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), None, None))


def _run(fn, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=fn, args=(r, world, port, q, *args)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    return sorted(out, key=lambda t: t[0])


@pytest.mark.parametrize("world", [2, 3])
def test_broadcast_gather(world):
    res = _run(_worker_collectives, world)
    for rank, same, order, mx in res:
        assert same is True, same
        assert order == [float(r) for r in range(world) for _ in range(2)]
        assert mx == 1.5 * (world - 1)


def _worker_sharded(rank, world, port, q):
    try:
        from deconv_api_amd.engine.deconvnet import DeconvNet
        from deconv_api_amd.models.vgg16 import VGG16, vgg16_specs
        from deconv_api_amd.parallel.sharded import ShardedRunner

        info = _init(rank, world, port)
        specs = vgg16_specs(width_div=8, image_size=32, fc=64, classes=10)
        eng = DeconvNet(VGG16.random(0, specs=specs).build("cpu", torch.float32))
        runner = ShardedRunner(eng, info, image_size=32)
        if rank == 0:
            rng = np.random.default_rng(0)
            imgs = [rng.integers(0, 256, (30 + i, 28, 3), dtype=np.uint8) for i in range(5)]  # ragged: 5 over 2
            out = runner.run("block3_conv2", imgs)
            out2 = runner.run("block1_pool", imgs[:1])
            runner.stop()
            single = ShardedRunner(eng, type(info)(), image_size=32)
            ref = single._prep(imgs)
            want = eng.run(ref, "block3_conv2", k=4).mosaic.numpy()
            q.put((rank, out.shape, bool(np.array_equal(out, want)), out2.shape))
        else:
            n = runner.follow()
            q.put((rank, n, None, None))
        from deconv_api_amd.parallel import dist as pdist

        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, traceback.format_exc(), None, None))


def test_sharded_deconv_matches_single():
    res = _run(_worker_sharded, 2)
    r0, r1 = res
    assert r0[1] == (5, 64, 64, 3), r0
    assert r0[2] is True
    assert r0[3] == (1, 64, 64, 3)
    assert r1[1] == 2, r1


def test_shard_sizes():
    from deconv_api_amd.parallel.dist import shard_counts, shard_sizes

    assert shard_sizes(2048, 8) == [256] * 8
    assert shard_sizes(5, 2) == [3, 3]
    assert shard_counts(5, 2) == [3, 2]
    assert sum(shard_counts(7, 4)) == 7
