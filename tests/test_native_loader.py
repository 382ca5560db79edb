"""Native record loader (``_native/loader.cpp``): exact transform vs a numpy reference using the
loader's own per-sample crop/flip parameters, epoch permutation determinism and independence of
the worker count, rank sharding, ring back-pressure, and the GPU path (pinned ring + async H2D)."""

import numpy as np
import pytest
import torch

from determined_amd.pytorch.native_loader import NativeImageLoader, _native, write_record_file


@pytest.fixture(scope="module")
def recfile(tmp_path_factory):
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, size=(37, 12, 10, 3), dtype=np.uint8)
    labels = np.arange(37) * 3 + 1
    p = tmp_path_factory.mktemp("rec") / "train.rec"
    write_record_file(str(p), imgs, labels)
    return str(p), imgs, labels


MEAN, STD = (0.5, 0.4, 0.3), (0.2, 0.25, 0.3)


def _ref(img, y0, x0, flip, ch, cw):
    crop = img[y0 : y0 + ch, x0 : x0 + cw].astype(np.float32)
    if flip:
        crop = crop[:, ::-1]
    return (crop / 255.0 - np.array(MEAN, np.float32)) / np.array(STD, np.float32)


def _collect(path, **kw):
    ld = NativeImageLoader(path, device="cpu", mean=MEAN, std=STD, **kw)
    out = [(x.clone(), y.clone()) for x, y in ld]
    return ld, out


def test_transform_exact_fp32(recfile):
    path, imgs, labels = recfile
    ld, out = _collect(path, batch_size=5, crop=(8, 6), dtype=torch.float32, seed=7, workers=3, drop_last=False)
    nat = _native()
    perm = nat.loader_permutation(37, 7, 0, True)
    assert sorted(perm) == list(range(37))
    assert len(out) == len(ld) == 8 and out[-1][0].shape[0] == 2
    k = 0
    for x, y in out:
        x = x.permute(0, 2, 3, 1).numpy()  # back to NHWC
        for i in range(x.shape[0]):
            idx = perm[k]
            y0, x0, flip = nat.loader_sample_params(7, 0, idx, 12, 10, 8, 6, True)
            np.testing.assert_allclose(x[i], _ref(imgs[idx], y0, x0, flip, 8, 6), rtol=1e-6, atol=1e-6)
            assert int(y[i]) == labels[idx]
            k += 1
    assert k == 37


def test_bf16_and_determinism_independent_of_workers(recfile):
    path, imgs, _ = recfile
    _, a = _collect(path, batch_size=4, crop=(12, 10), dtype=torch.bfloat16, seed=3, workers=1, augment=False)
    _, b = _collect(path, batch_size=4, crop=(12, 10), dtype=torch.bfloat16, seed=3, workers=6, augment=False,
                    prefetch=2)
    assert len(a) == 9  # drop_last
    for (xa, ya), (xb, yb) in zip(a, b):
        assert torch.equal(xa, xb) and torch.equal(ya, yb)
    perm = _native().loader_permutation(37, 3, 0, True)
    ref = torch.from_numpy(_ref(imgs[perm[0]], 0, 0, False, 12, 10)).to(torch.bfloat16)
    assert torch.equal(a[0][0][0].permute(1, 2, 0), ref)


def test_epochs_reshuffle_and_rank_sharding(recfile):
    path, _, labels = recfile
    ld = NativeImageLoader(path, batch_size=4, crop=(8, 8), device="cpu", seed=1, rank=0, world=1, drop_last=False)
    e0 = torch.cat([y for _, y in ld])
    e1 = torch.cat([y for _, y in ld])  # epoch advances automatically
    assert sorted(e0.tolist()) == sorted(e1.tolist()) == sorted(labels.tolist())
    assert e0.tolist() != e1.tolist()
    shards = []
    for r in range(3):
        ld = NativeImageLoader(path, batch_size=4, crop=(8, 8), device="cpu", seed=1, rank=r, world=3,
                               drop_last=True)
        shards.append(set(torch.cat([y for _, y in ld]).tolist()))
        assert len(shards[-1]) == 12  # 37 // 3 = 12 samples/rank, 3 batches of 4
    assert not (shards[0] & shards[1]) and not (shards[1] & shards[2]) and not (shards[0] & shards[2])


def test_bad_inputs(tmp_path, recfile):
    path, _, _ = recfile
    with pytest.raises(Exception):
        NativeImageLoader(path, batch_size=2, crop=(20, 20), device="cpu")
    bad = tmp_path / "bad.rec"
    bad.write_bytes(b"x" * 64)
    with pytest.raises(Exception):
        NativeImageLoader(str(bad), batch_size=2, crop=(8, 8), device="cpu")


@pytest.mark.gpu
def test_gpu_async_copy_matches_cpu(recfile):
    path, _, _ = recfile
    _, cpu = _collect(path, batch_size=8, crop=(8, 8), dtype=torch.bfloat16, seed=5)
    ld = NativeImageLoader(path, batch_size=8, crop=(8, 8), dtype=torch.bfloat16, seed=5, mean=MEAN, std=STD,
                           device="cuda", prefetch=2)
    gpu = [(x.float().sum(), x.clone(), y.clone()) for x, y in ld]
    torch.cuda.synchronize()
    assert len(gpu) == len(cpu)
    for (_, xg, yg), (xc, yc) in zip(gpu, cpu):
        assert xg.is_cuda and xg.is_contiguous(memory_format=torch.channels_last)
        assert torch.equal(xg.cpu(), xc) and torch.equal(yg.cpu(), yc)
