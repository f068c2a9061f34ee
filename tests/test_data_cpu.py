"""Real-data pipelines (data/real.py) on synthetic files in the raw on-disk
formats: CIFAR-10 binary batches, MNIST idx, PTB text, .npz arrays.
Reference: dl_trainer.py:295-502 (DistributedSampler per rank), ptb_reader.py."""
import os

import numpy as np
import torch

from gaussiank_sgd_amd.data import real


def _cifar(root, n_per=20):
    d = os.path.join(root, "cifar-10-batches-bin")
    os.makedirs(d)
    rng = np.random.default_rng(0)
    for name in ["data_batch_%d.bin" % i for i in range(1, 6)] + ["test_batch.bin"]:
        a = rng.integers(0, 256, size=(n_per, 3073), dtype=np.uint8)
        a[:, 0] = rng.integers(0, 10, size=n_per)
        a.tofile(os.path.join(d, name))


def _idx(path, arr):
    with open(path, "wb") as f:
        f.write(bytes([0, 0, 8, arr.ndim]))
        for s in arr.shape:
            f.write(int(s).to_bytes(4, "big"))
        f.write(arr.astype(np.uint8).tobytes())


def test_cifar10_reader_and_sharding(tmp_path):
    _cifar(str(tmp_path))
    x, y = real.read_cifar10_bin(str(tmp_path))
    assert x.shape == (100, 3, 32, 32) and x.dtype == torch.uint8 and y.max() < 10
    # DistributedSampler semantics: disjoint shards covering the set, new order each epoch
    shards = [real.ShardedSampler(100, 8, r, 4, seed=3).indices() for r in range(4)]
    allidx = torch.cat(shards)
    assert allidx.unique().numel() == 100 and all(s.numel() == 25 for s in shards)
    s = real.ShardedSampler(100, 8, 0, 4, seed=3)
    e0 = s.indices()
    s.set_epoch(1)
    assert not torch.equal(e0, s.indices())
    assert s.batches_per_epoch() == 3       # ragged last batch dropped


def test_device_loader_cifar_transform(tmp_path):
    _cifar(str(tmp_path))
    ld = real.open_dataset("cifar10", str(tmp_path), 16, "cpu", rank=1, world=2, seed=0)
    xb, yb = next(ld)
    assert xb.shape == (16, 3, 32, 32) and xb.dtype == torch.float32 and yb.shape == (16,)
    assert abs(float(xb.mean())) < 1.0            # normalised
    # epochs roll over forever (data_iter semantics)
    for _ in range(2 * ld.batches_per_epoch() + 1):
        next(ld)
    assert ld.epoch >= 2
    ld.close()


def test_mnist_idx_and_npz(tmp_path):
    rng = np.random.default_rng(1)
    _idx(str(tmp_path / "train-images-idx3-ubyte"), rng.integers(0, 256, (50, 28, 28)))
    _idx(str(tmp_path / "train-labels-idx1-ubyte"), rng.integers(0, 10, (50,)))
    x, y = real.read_mnist_idx(str(tmp_path))
    assert x.shape == (50, 1, 28, 28) and y.shape == (50,)
    np.savez(str(tmp_path / "imagenet_train.npz"), x=rng.integers(0, 256, (12, 3, 40, 40), dtype=np.uint8),
             y=rng.integers(0, 1000, (12,)))
    ld = real.open_dataset("imagenet", str(tmp_path), 4, "cpu", image_size=32)
    xb, yb = next(ld)
    assert xb.shape == (4, 3, 32, 32) and yb.dtype == torch.int64
    ld.close()


def test_ptb_vocab_and_windows(tmp_path):
    txt = " the cat sat \n the dog sat on the mat \n"   # PTB lines: space-padded
    for split in ("train", "valid", "test"):
        (tmp_path / ("ptb.%s.txt" % split)).write_text(txt * 20)
    tr, va, te, w2i, i2w = real.ptb_raw_data(str(tmp_path))
    # descending frequency, ties alphabetical (ptb_reader.py:14-24)
    assert i2w[0] == "the" and w2i["<eos>"] < w2i["cat"]
    x, y = real.ptb_windows(tr, 5, 4)
    assert torch.equal(x[:, 1:], y[:, :-1])
    ld = real.open_dataset("ptb", str(tmp_path), 4, "cpu", num_steps=5)
    xb, yb = next(ld)
    assert xb.shape == (5, 4)                       # [T, B] like the model input
    ld.close()


def test_trainer_uses_real_data(tmp_path):
    from gaussiank_sgd_amd.train import DLTrainer
    _cifar(str(tmp_path))
    t = DLTrainer(0, 2, dnn="resnet20", dataset="cifar10", batch_size=8, device="cpu", data_dir=str(tmp_path),
                  nworkers=2)
    assert isinstance(t.data, real.DeviceLoader) and t.trainset_len == 100
    t.train(1)
    t.data.close()


def _jpeg_tree(root, classes=3, per_class=5):
    from PIL import Image
    rng = np.random.default_rng(0)
    for split in ("train", "val"):
        for c in range(classes):
            d = root / split / ("n%08d" % c)
            d.mkdir(parents=True)
            for i in range(per_class):
                w, h = int(rng.integers(40, 90)), int(rng.integers(40, 90))
                arr = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
                Image.fromarray(arr).save(str(d / ("img_%d.JPEG" % i)), quality=90)


def test_imagenet_image_folder_loader(tmp_path):
    """ImageNet image-folder reader: class labels from sorted sub-directories,
    RandomResizedCrop + flip on the host (train) / Resize + CenterCrop (eval),
    rank sharding with DistributedSampler semantics, GPU-side normalisation
    (here: CPU), reproducible crops."""
    _jpeg_tree(tmp_path)
    S = 32
    loaders = [real.open_dataset("imagenet", str(tmp_path), 4, "cpu", rank=r, world=2, seed=3, image_size=S)
               for r in range(2)]
    for ld in loaders:
        assert ld is not None and ld.num_samples() == 15
        assert ld.sampler.per_rank == 8 and ld.batches_per_epoch() == 2
        x, y = next(ld)
        assert x.shape == (4, 3, S, S) and x.dtype == torch.float32
        assert y.dtype == torch.int64 and int(y.min()) >= 0 and int(y.max()) <= 2
        assert float(x.abs().max()) < 3.0 / 0.224          # normalised
        ld.close()
    # the two ranks see disjoint sample sets in an epoch (15 samples padded to 16)
    idx = [set(real.ShardedSampler(15, 4, r, 2, seed=3).indices().tolist()) for r in range(2)]
    assert len(idx[0] | idx[1]) == 15
    # crops are a pure function of (seed, epoch, index)
    rows = real.ImageFolderRows(real.find_image_folder(str(tmp_path), True), S, True, seed=5)
    a, b = rows.load(3), rows.load(3)
    assert a.shape == (3, S, S) and np.array_equal(a, b)
    rows.set_epoch(1)
    assert not np.array_equal(rows.load(3), a)
    ev = real.open_dataset("imagenet", str(tmp_path), 5, "cpu", train=False, image_size=S)
    xe, ye = next(ev)
    assert xe.shape == (5, 3, S, S) and ye.tolist() == [0, 0, 0, 0, 0]     # eval: not shuffled
    ev.close()
    l, t, w, h = real.random_resized_crop_box(100, 60, np.random.default_rng(1))
    assert 0 <= l and l + w <= 100 and 0 <= t and t + h <= 60
