"""CIFAR-10 readers (no torchvision, no network).

The reference reads ``torchvision.datasets.CIFAR10(root=--data-dir)`` and downloads it on
rank 0 (reference train_ddp.py:103-119).  The GPU box has no network, so this reader only
uses files already present under ``--data-dir``:

* ``cifar-10-batches-bin/{data_batch_1..5,test_batch}.bin`` - the raw binary release
  (1 label byte + 3072 pixel bytes per record), read with numpy, nothing executed;
* ``cifar-10-batches-py/{data_batch_1..5,test_batch}`` - the python release, read with a
  *restricted* unpickler that only admits the numpy array reconstruction globals the
  files legitimately use (no arbitrary code execution from a data file).

Images come back as uint8 ``[N, 3, 32, 32]`` (CHW, the files' native order) plus int64
labels; the device loader keeps them resident in HBM and augments on the GPU.
"""
from __future__ import annotations

import io
import pickle
from pathlib import Path
from typing import Optional, Tuple

import numpy as np

TRAIN_BATCHES = [f"data_batch_{i}" for i in range(1, 6)]
TEST_BATCHES = ["test_batch"]
MEAN = (0.4914, 0.4822, 0.4465)
STD = (0.2470, 0.2435, 0.2616)


class _SafeUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"),
        ("numpy._core.multiarray", "_reconstruct"),
        ("numpy", "ndarray"),
        ("numpy", "dtype"),
        ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"),
        ("_codecs", "encode"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"CIFAR reader refuses global {module}.{name}")


def _read_py_batch(path: Path) -> Tuple[np.ndarray, np.ndarray]:
    with open(path, "rb") as f:
        d = _SafeUnpickler(io.BytesIO(f.read()), encoding="bytes").load()
    data = d.get(b"data", d.get("data"))
    labels = d.get(b"labels", d.get("labels"))
    x = np.asarray(data, dtype=np.uint8).reshape(-1, 3, 32, 32)
    return x, np.asarray(labels, dtype=np.int64)


def _read_bin_batch(path: Path) -> Tuple[np.ndarray, np.ndarray]:
    raw = np.fromfile(path, dtype=np.uint8)
    if raw.size % 3073:
        raise ValueError(f"{path}: not a CIFAR-10 binary batch")
    rec = raw.reshape(-1, 3073)
    return rec[:, 1:].reshape(-1, 3, 32, 32).copy(), rec[:, 0].astype(np.int64)


def find_cifar10(root: str) -> Optional[Tuple[str, Path]]:
    r = Path(root)
    for kind, sub in (("bin", "cifar-10-batches-bin"), ("py", "cifar-10-batches-py")):
        d = r / sub
        if d.is_dir() and all(((d / (b + ".bin")) if kind == "bin" else (d / b)).exists()
                              for b in TRAIN_BATCHES + TEST_BATCHES):
            return kind, d
    return None


def load_cifar10(root: str, train: bool) -> Tuple[np.ndarray, np.ndarray]:
    found = find_cifar10(root)
    if found is None:
        raise FileNotFoundError(
            f"CIFAR-10 not found under {root!r} (expected cifar-10-batches-bin/ or "
            "cifar-10-batches-py/). There is no network to download it: place the files there "
            "or use --dataset synthetic.")
    kind, d = found
    names = TRAIN_BATCHES if train else TEST_BATCHES
    xs, ys = [], []
    for b in names:
        x, y = _read_bin_batch(d / (b + ".bin")) if kind == "bin" else _read_py_batch(d / b)
        xs.append(x)
        ys.append(y)
    return np.concatenate(xs), np.concatenate(ys)
