"""Real-data pipelines with rank sharding (``--data-dir``).

Parity: reference dl_trainer.py:295-502 (CIFAR-10 / MNIST via torchvision,
ImageNet via HDF5, PTB via ptb_reader.py:9-102, AN4), each behind a
``DistributedSampler(num_replicas=nworkers, rank=rank)`` and a single-threaded
DataLoader (its IO was ~30% of an iteration).

MI355X design:
  * storage readers parse the raw on-disk formats directly -- CIFAR-10 binary
    batches, MNIST idx files, PTB text, ``.npy``/``.npz`` arrays (numpy with
    ``allow_pickle=False``; large arrays are memory-mapped) -- nothing is
    unpickled and nothing is downloaded;
  * ``ShardedSampler`` = DistributedSampler semantics (padded to a multiple of
    the world size, rank-strided, reshuffled every epoch from seed + epoch,
    ragged last batch dropped as the reference's data_iter does);
  * ``DeviceLoader`` keeps uint8 images on the host, gathers each batch with a
    background thread into pinned memory, copies it to the GPU on a side
    stream (non_blocking) and runs normalisation / augmentation ON THE GPU
    (random crop + flip + normalise as one batched op), so the training
    stream never waits for the host;
  * ImageNet as an image folder (``<root>/train/<class>/*.JPEG``, torchvision
    ImageFolder layout; the reference's HDF5 reader is broken):
    ``ImageFolderRows`` decodes with PIL in a thread pool inside the
    loader's gather thread and applies the reference's host transform --
    ``RandomResizedCrop(224)`` + horizontal flip for training, ``Resize(256)``
    + ``CenterCrop(224)`` for evaluation (dl_trainer.py:305-313) -- to uint8;
    the normalisation runs on the GPU.
"""
from __future__ import annotations

import collections
import os
import queue
import threading
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch

CIFAR_MEAN, CIFAR_STD = (0.491, 0.482, 0.447), (0.247, 0.243, 0.262)      # dl_trainer.py:348
MNIST_MEAN, MNIST_STD = (0.1307,), (0.3081,)                             # dl_trainer.py:390
IMAGENET_MEAN, IMAGENET_STD = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)


# ---------------------------------------------------------------------------
# readers
# ---------------------------------------------------------------------------
def read_cifar10_bin(root: str, train: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """CIFAR-10 binary version (``cifar-10-batches-bin/data_batch_{1..5}.bin``,
    ``test_batch.bin``): records of 1 label byte + 3072 pixel bytes (CHW)."""
    d = root
    if os.path.isdir(os.path.join(root, "cifar-10-batches-bin")):
        d = os.path.join(root, "cifar-10-batches-bin")
    names = ["data_batch_%d.bin" % i for i in range(1, 6)] if train else ["test_batch.bin"]
    raw = [np.fromfile(os.path.join(d, n), dtype=np.uint8).reshape(-1, 3073) for n in names]
    a = np.concatenate(raw, 0)
    y = torch.from_numpy(a[:, 0].astype(np.int64))
    x = torch.from_numpy(np.ascontiguousarray(a[:, 1:]).reshape(-1, 3, 32, 32))
    return x, y


def _read_idx(path: str) -> np.ndarray:
    with open(path, "rb") as f:
        data = f.read()
    magic = int.from_bytes(data[0:4], "big")
    ndim = magic & 0xFF
    dims = [int.from_bytes(data[4 + 4 * i:8 + 4 * i], "big") for i in range(ndim)]
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * ndim).reshape(dims)


def read_mnist_idx(root: str, train: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """MNIST idx files (``train-images-idx3-ubyte`` / ``t10k-...``, optionally under MNIST/raw)."""
    for d in (root, os.path.join(root, "MNIST", "raw"), os.path.join(root, "raw")):
        pre = "train" if train else "t10k"
        img = os.path.join(d, "%s-images-idx3-ubyte" % pre)
        lab = os.path.join(d, "%s-labels-idx1-ubyte" % pre)
        if os.path.isfile(img) and os.path.isfile(lab):
            x = torch.from_numpy(_read_idx(img).copy()).unsqueeze(1)
            y = torch.from_numpy(_read_idx(lab).astype(np.int64))
            return x, y
    raise FileNotFoundError("no MNIST idx files under %s" % root)


def load_arrays(path: str, mmap: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """``x``/``y`` from an ``.npz`` (keys x, y) or a pair ``<path>_x.npy`` / ``<path>_y.npy``
    (memory-mapped, for ImageNet-sized uint8 image arrays)."""
    if path.endswith(".npz"):
        d = np.load(path, allow_pickle=False)
        return torch.from_numpy(np.asarray(d["x"])), torch.from_numpy(np.asarray(d["y"]).astype(np.int64))
    base = path[:-6] if path.endswith("_x.npy") else path
    x = np.load(base + "_x.npy", mmap_mode="r" if mmap else None, allow_pickle=False)
    y = np.load(base + "_y.npy", allow_pickle=False).astype(np.int64)
    return torch.from_numpy(np.asarray(x)) if not mmap else _MmapRows(x), torch.from_numpy(y)


class _MmapRows:
    """Row view of a memory-mapped numpy array: gathers only the rows a batch needs."""

    def __init__(self, arr: np.ndarray):
        self.arr = arr
        self.shape = arr.shape
        self.dtype = torch.from_numpy(np.zeros(1, dtype=arr.dtype)).dtype

    def __len__(self):
        return self.shape[0]

    def gather(self, idx: torch.Tensor, out: torch.Tensor) -> None:
        ii = np.sort(idx.numpy())          # sequential reads; order restored below
        order = np.argsort(np.argsort(idx.numpy()))
        rows = self.arr[ii][order]
        out.copy_(torch.from_numpy(np.ascontiguousarray(rows)))


# ---------------------------------------------------------------------------
# PTB (ptb_reader.py:9-102)
# ---------------------------------------------------------------------------
def _read_words(path: str) -> List[str]:
    with open(path, "r") as f:
        return f.read().replace("\n", "<eos>").split()


IMAGE_EXTS = (".jpg", ".jpeg", ".png", ".bmp", ".ppm", ".webp")


def find_image_folder(root: str, train: bool = True) -> Optional[str]:
    """``root/train`` (``root/val``) when present, else ``root`` itself, if it
    holds class sub-directories with images."""
    for cand in ([os.path.join(root, "train")] if train else [os.path.join(root, "val"), os.path.join(root, "test")]) + [root]:
        if os.path.isdir(cand):
            subs = [d for d in sorted(os.listdir(cand)) if os.path.isdir(os.path.join(cand, d))]
            if subs and any(f.lower().endswith(IMAGE_EXTS) for f in os.listdir(os.path.join(cand, subs[0]))):
                return cand
    return None


def scan_image_folder(folder: str) -> Tuple[List[str], torch.Tensor, List[str]]:
    """(files, labels, classes): classes = sorted sub-directory names, label =
    class index (torchvision ImageFolder convention)."""
    classes = sorted(d for d in os.listdir(folder) if os.path.isdir(os.path.join(folder, d)))
    files, labels = [], []
    for ci, c in enumerate(classes):
        cdir = os.path.join(folder, c)
        for f in sorted(os.listdir(cdir)):
            if f.lower().endswith(IMAGE_EXTS):
                files.append(os.path.join(cdir, f))
                labels.append(ci)
    return files, torch.tensor(labels, dtype=torch.int64), classes


def random_resized_crop_box(W: int, H: int, rng: np.random.Generator, scale=(0.08, 1.0),
                            ratio=(3.0 / 4.0, 4.0 / 3.0)) -> Tuple[int, int, int, int]:
    """torchvision RandomResizedCrop.get_params: (left, top, width, height)."""
    import math
    area = H * W
    log_r = (math.log(ratio[0]), math.log(ratio[1]))
    for _ in range(10):
        target = area * rng.uniform(scale[0], scale[1])
        ar = math.exp(rng.uniform(log_r[0], log_r[1]))
        w = int(round(math.sqrt(target * ar)))
        h = int(round(math.sqrt(target / ar)))
        if 0 < w <= W and 0 < h <= H:
            top = int(rng.integers(0, H - h + 1))
            left = int(rng.integers(0, W - w + 1))
            return left, top, w, h
    in_ratio = float(W) / float(H)   # fallback: centre crop at the clamped ratio
    if in_ratio < min(ratio):
        w, h = W, int(round(W / min(ratio)))
    elif in_ratio > max(ratio):
        h, w = H, int(round(H * max(ratio)))
    else:
        w, h = W, H
    return (W - w) // 2, (H - h) // 2, w, h


class ImageFolderRows:
    """An image folder as rows of uint8 [3, size, size] images, decoded on
    demand (``gather``) with the reference's train / eval host transforms.
    Randomness is a pure function of (seed, epoch, sample index), so every
    rank's crops are reproducible and independent of the thread schedule."""

    def __init__(self, folder: str, size: int = 224, train: bool = True, seed: int = 0, workers: int = 8):
        self.files, self.labels, self.classes = scan_image_folder(folder)
        if not self.files:
            raise OSError("no images under %s" % folder)
        self.size, self.train, self.seed = int(size), bool(train), int(seed)
        self.shape = (len(self.files), 3, self.size, self.size)
        self.dtype = torch.uint8
        self.epoch = 0
        self._pool = None
        self._workers = max(1, int(workers))

    def __len__(self) -> int:
        return len(self.files)

    def load(self, i: int) -> np.ndarray:
        from PIL import Image
        with Image.open(self.files[i]) as im:
            im = im.convert("RGB")
            S = self.size
            if self.train:
                rng = np.random.default_rng((self.seed, self.epoch, int(i)))
                left, top, w, h = random_resized_crop_box(im.width, im.height, rng)
                im = im.resize((S, S), Image.BILINEAR, box=(left, top, left + w, top + h))
                if rng.random() < 0.5:
                    im = im.transpose(Image.FLIP_LEFT_RIGHT)
            else:
                short = int(round(S * 256 / 224))          # Resize(256) for 224 crops
                if im.width <= im.height:
                    nw, nh = short, int(short * im.height / im.width)
                else:
                    nw, nh = int(short * im.width / im.height), short
                im = im.resize((nw, nh), Image.BILINEAR)
                left, top = int(round((nw - S) / 2.0)), int(round((nh - S) / 2.0))
                im = im.crop((left, top, left + S, top + S))
            return np.asarray(im, dtype=np.uint8).transpose(2, 0, 1)

    def gather(self, idx: torch.Tensor, out: torch.Tensor) -> None:
        import concurrent.futures as cf
        if self._pool is None:
            self._pool = cf.ThreadPoolExecutor(max_workers=self._workers, thread_name_prefix="gk-decode")
        ids = [int(i) for i in idx.tolist()]
        for b, arr in enumerate(self._pool.map(self.load, ids)):
            out[b].copy_(torch.from_numpy(arr))

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)


def ptb_raw_data(data_path: str, prefix: str = "ptb"):
    """(train, valid, test, word_to_id, id_to_word): vocabulary by descending
    frequency, ties alphabetical, from the training file (ptb_reader.py:14-52)."""
    train_path = os.path.join(data_path, prefix + ".train.txt")
    words = _read_words(train_path)
    counter = collections.Counter(words)
    pairs = sorted(counter.items(), key=lambda x: (-x[1], x[0]))
    word_to_id = {w: i for i, (w, _) in enumerate(pairs)}
    id_to_word = {i: w for w, i in word_to_id.items()}

    def ids(p):
        return [word_to_id[w] for w in _read_words(p) if w in word_to_id]
    return (ids(train_path), ids(os.path.join(data_path, prefix + ".valid.txt")),
            ids(os.path.join(data_path, prefix + ".test.txt")), word_to_id, id_to_word)


def ptb_windows(token_ids, num_steps: int, batch_size: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """TrainDataset windows (ptb_reader.py:55-79): sample i = ids[T*i : T*i+T] and
    the next-token targets; length rounded down to a multiple of batch_size."""
    raw = torch.tensor(token_ids, dtype=torch.int64)
    n = (raw.numel() - 1) // num_steps
    n -= n % batch_size
    x = raw[: n * num_steps].view(n, num_steps)
    y = raw[1: n * num_steps + 1].view(n, num_steps)
    return x, y


# ---------------------------------------------------------------------------
# sampling
# ---------------------------------------------------------------------------
class ShardedSampler:
    """DistributedSampler semantics: pad to a multiple of the world, stride by
    rank, permutation from (seed + epoch); drop the ragged last batch."""

    def __init__(self, n: int, batch_size: int, rank: int = 0, world: int = 1, seed: int = 0, shuffle: bool = True):
        self.n, self.bs, self.rank, self.world = int(n), int(batch_size), int(rank), max(1, int(world))
        self.seed, self.shuffle = int(seed), shuffle
        self.epoch = 0
        self.per_rank = (self.n + self.world - 1) // self.world

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def indices(self) -> torch.Tensor:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            perm = torch.randperm(self.n, generator=g)
        else:
            perm = torch.arange(self.n)
        total = self.per_rank * self.world
        if total > self.n:
            perm = torch.cat([perm, perm[: total - self.n]])
        return perm[self.rank:total:self.world]

    def batches_per_epoch(self) -> int:
        return self.per_rank // self.bs

    def __iter__(self):
        idx = self.indices()
        for b in range(self.batches_per_epoch()):
            yield idx[b * self.bs:(b + 1) * self.bs]


# ---------------------------------------------------------------------------
# GPU-side transforms (batched)
# ---------------------------------------------------------------------------
def normalize_transform(mean, std, channels_last: bool = False):
    def fn(x: torch.Tensor, train: bool) -> torch.Tensor:
        m = torch.tensor(mean, device=x.device, dtype=torch.float32).view(1, -1, 1, 1)
        s = torch.tensor(std, device=x.device, dtype=torch.float32).view(1, -1, 1, 1)
        y = (x.float() * (1.0 / 255.0) - m) / s
        return y.contiguous(memory_format=torch.channels_last) if channels_last else y
    return fn


def crop_flip_transform(mean, std, size: int, pad: int = 0, channels_last: bool = False, seed: int = 0):
    """Random crop (``pad`` zero padding, or a random ``size`` window of a larger
    stored image) + random horizontal flip + normalise, on the device, for the
    whole batch at once (RandomCrop / RandomHorizontalFlip / Normalize of
    dl_trainer.py:349-353).  Evaluation: centre crop."""
    gen: Dict[torch.device, torch.Generator] = {}

    def fn(x: torch.Tensor, train: bool) -> torch.Tensor:
        B, C, H, W = x.shape
        xf = x.float() * (1.0 / 255.0)
        if pad:
            xf = torch.nn.functional.pad(xf, (pad, pad, pad, pad))
            H, W = H + 2 * pad, W + 2 * pad
        dev = x.device
        if train:
            g = gen.get(dev)
            if g is None:
                g = torch.Generator(device=dev)
                g.manual_seed(seed)
                gen[dev] = g
            oy = torch.randint(0, H - size + 1, (B,), device=dev, generator=g)
            ox = torch.randint(0, W - size + 1, (B,), device=dev, generator=g)
            flip = torch.rand(B, device=dev, generator=g) < 0.5
        else:
            oy = torch.full((B,), (H - size) // 2, device=dev)
            ox = torch.full((B,), (W - size) // 2, device=dev)
            flip = torch.zeros(B, dtype=torch.bool, device=dev)
        ar = torch.arange(size, device=dev)
        rows = (oy[:, None] + ar[None, :])                                   # [B, size]
        cols = (ox[:, None] + ar[None, :])
        cols = torch.where(flip[:, None], cols.flip(1), cols)
        bi = torch.arange(B, device=dev)[:, None, None]
        out = xf.permute(0, 2, 3, 1)[bi, rows[:, :, None], cols[:, None, :]]  # [B, size, size, C]
        m = torch.tensor(mean, device=dev, dtype=torch.float32)
        s = torch.tensor(std, device=dev, dtype=torch.float32)
        out = (out - m) / s
        out = out.permute(0, 3, 1, 2)
        return out if channels_last else out.contiguous()
    return fn


# ---------------------------------------------------------------------------
# loader
# ---------------------------------------------------------------------------
class DeviceLoader:
    """Sharded, prefetching batch iterator over host arrays.

    A background thread gathers the next ``prefetch`` batches into pinned
    buffers; each is copied to the device on a side stream and handed over
    with an event, then ``transform`` (GPU) makes the model input.  Iteration
    never ends: at the end of an epoch the sampler advances to the next epoch
    (new permutation), like the reference's data_iter restarting its loader."""

    def __init__(self, x, y, batch_size: int, device="cpu", rank: int = 0, world: int = 1, seed: int = 0,
                 transform: Optional[Callable] = None, train: bool = True, prefetch: int = 2,
                 shuffle: bool = True, seq_first: bool = False):
        self.x, self.y = x, y
        self.device = torch.device(device)
        self.sampler = ShardedSampler(x.shape[0], batch_size, rank, world, seed, shuffle)
        self.transform = transform
        self.train = train
        self.seq_first = seq_first
        self.batch_size = int(batch_size)
        self.epoch = 0
        self._pin = self.device.type == "cuda"
        self._stream = torch.cuda.Stream(self.device) if self._pin else None
        self._q: "queue.Queue" = queue.Queue(maxsize=max(1, prefetch))
        self._stop = threading.Event()
        # the prefetch thread starts on the first next(): an evaluation split
        # that is only walked by full_pass() never runs one
        self._thread: Optional[threading.Thread] = None

    def num_samples(self) -> int:
        return self.sampler.n

    def batches_per_epoch(self) -> int:
        return self.sampler.batches_per_epoch()

    def _gather(self, idx: torch.Tensor):
        xs = (idx.numel(),) + tuple(self.x.shape[1:])
        xb = torch.empty(xs, dtype=self.x.dtype, pin_memory=self._pin)
        if isinstance(self.x, (_MmapRows, ImageFolderRows)):   # memory-mapped arrays, decoded image folders
            self.x.gather(idx, xb)
        else:
            torch.index_select(self.x, 0, idx, out=xb)
        yb = torch.empty((idx.numel(),) + tuple(self.y.shape[1:]), dtype=self.y.dtype, pin_memory=self._pin)
        torch.index_select(self.y, 0, idx, out=yb)
        return xb, yb

    def _producer(self):
        try:
            while not self._stop.is_set():
                for idx in self.sampler:
                    if self._stop.is_set():
                        return
                    self._q.put(self._gather(idx))
                self.epoch += 1
                self.sampler.set_epoch(self.epoch)
                if isinstance(self.x, ImageFolderRows):
                    self.x.set_epoch(self.epoch)
        except BaseException as e:  # noqa: BLE001 - surfaced on the consumer side
            self._q.put(e)

    def __iter__(self):
        return self

    def __next__(self):
        if self._thread is None:
            self._thread = threading.Thread(target=self._producer, name="gk-data", daemon=True)
            self._thread.start()
        item = self._q.get()
        if isinstance(item, BaseException):
            raise item
        return self._deliver(*item)

    def _deliver(self, xb: torch.Tensor, yb: torch.Tensor):
        if self._stream is not None:
            with torch.cuda.stream(self._stream):
                xd = xb.to(self.device, non_blocking=True)
                yd = yb.to(self.device, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._stream)
            torch.cuda.current_stream(self.device).wait_event(ev)
            xd.record_stream(torch.cuda.current_stream(self.device))
            yd.record_stream(torch.cuda.current_stream(self.device))
        else:
            xd, yd = xb, yb
        if self.transform is not None:
            xd = self.transform(xd, self.train)
        if self.seq_first:
            xd, yd = xd.t().contiguous(), yd.t().contiguous()
        return xd, yd

    def close(self) -> None:
        self._stop.set()
        try:
            while True:
                self._q.get_nowait()
        except queue.Empty:
            pass

    def test_batches(self, n: int = 2):
        return [next(self) for _ in range(n)]

    def full_pass(self):
        """Every sample of the split exactly once, in storage order, in
        batches of ``batch_size`` with the ragged last batch INCLUDED -- the
        reference's ``testloader`` (DataLoader(shuffle=False), drop_last
        False; dl_trainer.py:339-342,376-377,753) that ``test()`` walks whole.
        Synchronous (no prefetch thread), independent of the training stream
        of batches."""
        n = self.sampler.n
        for s in range(0, n, self.batch_size):
            idx = torch.arange(s, min(n, s + self.batch_size))
            yield self._deliver(*self._gather(idx))


def open_dataset(dataset: str, data_dir: str, batch_size: int, device, rank: int = 0, world: int = 1,
                 seed: int = 0, channels_last: bool = False, num_steps: int = 35, train: bool = True,
                 image_size: Optional[int] = None) -> Optional[DeviceLoader]:
    """A DeviceLoader over the real data in ``data_dir`` for ``dataset``, or None
    when the directory holds no recognised files (the caller falls back to
    synthetic data and says so)."""
    if not data_dir or not os.path.isdir(data_dir):
        return None
    split = "train" if train else "test"
    npz = os.path.join(data_dir, "%s_%s.npz" % (dataset, split))
    npy = os.path.join(data_dir, "%s_%s" % (dataset, split))
    x = y = None
    if os.path.isfile(npz):
        x, y = load_arrays(npz)
    elif os.path.isfile(npy + "_x.npy"):
        x, y = load_arrays(npy)
    elif dataset == "cifar10":
        try:
            x, y = read_cifar10_bin(data_dir, train)
        except OSError:
            return None
    elif dataset in ("mnist", "mnist32"):
        try:
            x, y = read_mnist_idx(data_dir, train)
        except OSError:
            return None
    elif dataset == "imagenet" and find_image_folder(data_dir, train) is not None:
        # image folder: host decode + the reference's crop / flip, GPU normalise
        rows = ImageFolderRows(find_image_folder(data_dir, train), image_size or 224, train, seed + 7919 * rank)
        return DeviceLoader(rows, rows.labels, batch_size, device, rank, world, seed,
                            normalize_transform(IMAGENET_MEAN, IMAGENET_STD, channels_last), train, shuffle=train)
    elif dataset == "ptb":
        if not os.path.isfile(os.path.join(data_dir, "ptb.train.txt")):
            return None
        tr, va, te, w2i, _ = ptb_raw_data(data_dir)
        # evaluation on the validation split, as the reference's test() does
        # (dl_trainer.py ptb_prepare: TestDataset(valid_data, ...))
        x, y = ptb_windows(tr if train else va, num_steps, batch_size)
        return DeviceLoader(x, y, batch_size, device, rank, world, seed, None, train, shuffle=train, seq_first=True)
    if x is None:
        return None
    if dataset == "cifar10":
        tf = crop_flip_transform(CIFAR_MEAN, CIFAR_STD, 32, pad=4, channels_last=channels_last, seed=seed + rank) \
            if train else normalize_transform(CIFAR_MEAN, CIFAR_STD, channels_last)
    elif dataset in ("mnist", "mnist32"):
        tf = normalize_transform(MNIST_MEAN, MNIST_STD, channels_last)
        if dataset == "mnist32" and x.shape[-1] == 28:
            x = torch.nn.functional.pad(x, (2, 2, 2, 2))
    elif dataset == "imagenet":
        size = image_size or 224
        tf = crop_flip_transform(IMAGENET_MEAN, IMAGENET_STD, size, 0, channels_last, seed=seed + rank)
    else:
        tf = None
    return DeviceLoader(x, y, batch_size, device, rank, world, seed, tf, train, shuffle=train)
