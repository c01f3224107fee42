"""Helpers for the -m gpu tests: numpy <-> device byte buffers (torch is plumbing only)."""
import numpy as np
import torch

DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def to_dev(a):
    """numpy array -> device byte tensor holding the same bytes."""
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(DEV)


def empty_dev(nbytes):
    return torch.zeros(max(int(nbytes), 1), dtype=torch.uint8, device=DEV)


def from_dev(t, npdt, n=None):
    raw = t.cpu().numpy()
    isz = np.dtype(npdt).itemsize
    a = raw[: raw.size - raw.size % isz].view(npdt)
    return a if n is None else a[:n]


def stream():
    return torch.cuda.current_stream(DEV)


def sync():
    torch.cuda.synchronize(DEV)
