"""Frame ingest: dataset PNGs -> pinned host batches -> HBM.

The reference reads one frame per step with cv2.imread(path, IMREAD_GRAYSCALE)
(utils.py:55-81).  Here libvo_ingest.so decodes a whole batch (one frame per chain) on a
pool of host threads into pinned memory, a Python thread keeps one batch ahead of the
consumer, and the host->HBM copy runs on its own stream, so decoding and the copy overlap
the GPU step of the previous batch.
"""
from __future__ import annotations

import ctypes as C
import os
import queue
import threading

import numpy as np
import torch

from . import _lib

_HERE = os.path.dirname(os.path.abspath(__file__))
INGEST_PATH = os.path.join(_HERE, "_build", "libvo_ingest.so")
_ing = None
_SYMS = ("vo_png_info", "vo_png_decode_gray", "vo_ingest_create", "vo_ingest_destroy", "vo_ingest_png_files")


def lib():
    global _ing
    if _ing is None:
        if not os.path.exists(INGEST_PATH):
            _lib.build()
        L = C.CDLL(INGEST_PATH)
        P, I, S = C.c_void_p, C.c_int, C.c_size_t
        L.vo_png_info.argtypes = [P, S, C.POINTER(I), C.POINTER(I), C.POINTER(I), C.POINTER(I)]
        L.vo_png_decode_gray.argtypes = [P, S, P, C.c_int64, I, I]
        L.vo_ingest_create.argtypes = [I]
        L.vo_ingest_create.restype = P
        L.vo_ingest_destroy.argtypes = [P]
        L.vo_ingest_destroy.restype = None
        L.vo_ingest_png_files.argtypes = [P, C.POINTER(C.c_char_p), I, P, C.c_int64, I, I, P]
        for n in ("vo_png_info", "vo_png_decode_gray", "vo_ingest_png_files"):
            getattr(L, n).restype = C.c_int
        _ing = L
    return _ing


def png_info(data: bytes):
    w, h, c, d = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    rc = lib().vo_png_info(data, len(data), C.byref(w), C.byref(h), C.byref(c), C.byref(d))
    if rc:
        raise ValueError(f"not a supported PNG (code {rc})")
    return w.value, h.value, c.value, d.value


def imread_gray(path: str) -> np.ndarray:
    """cv2.imread(path, cv2.IMREAD_GRAYSCALE) for PNG files (utils.py:59,81)."""
    with open(path, "rb") as f:
        data = f.read()
    w, h, _, _ = png_info(data)
    out = np.empty((h, w), np.uint8)
    rc = lib().vo_png_decode_gray(data, len(data), out.ctypes.data, w, w, h)
    if rc:
        raise ValueError(f"{path}: PNG decode failed (code {rc})")
    return out


class FrameSource:
    """Iterate over batches of PNG paths (batches[j][b] = frame of chain b at step j) and yield
    uint8 [B, H, W] tensors on `device`, decoded one batch ahead of the consumer."""

    def __init__(self, batches, width: int, height: int, device="cuda", threads: int = 8, depth: int = 2):
        self.batches = [list(b) for b in batches]
        self.W, self.H = int(width), int(height)
        self.device = torch.device(device)
        self.B = len(self.batches[0]) if self.batches else 0
        gpu = self.device.type == "cuda"
        self._bufs = [torch.empty((self.B, self.H, self.W), dtype=torch.uint8, pin_memory=gpu)
                      for _ in range(max(2, depth))]
        self._free = queue.Queue()
        for i in range(len(self._bufs)):
            self._free.put(i)
        self._ready = queue.Queue()
        self._pool = lib().vo_ingest_create(int(threads))
        self._copy_stream = torch.cuda.Stream(self.device) if gpu else None
        self._thread = threading.Thread(target=self._decode_all, daemon=True)
        self._thread.start()

    def _decode_all(self):
        L = lib()
        for j, paths in enumerate(self.batches):
            slot = self._free.get()
            if slot is None:
                return
            arr = (C.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
            st = np.zeros(len(paths), np.int32)
            rc = L.vo_ingest_png_files(self._pool, arr, len(paths), self._bufs[slot].data_ptr(),
                                       self.H * self.W, self.W, self.H, st.ctypes.data)
            self._ready.put((j, slot, rc, st))
        self._ready.put(None)

    def __len__(self):
        return len(self.batches)

    def __iter__(self):
        pending = None                                   # (event, slot) of the last copy
        while True:
            item = self._ready.get()
            if item is None:
                break
            j, slot, rc, st = item
            if rc:
                bad = [self.batches[j][i] for i in np.nonzero(st)[0][:3]]
                raise RuntimeError(f"frame decode failed for {bad} (codes {st[st != 0][:3].tolist()})")
            if self._copy_stream is None:
                out = self._bufs[slot].clone()
                self._free.put(slot)
            else:
                with torch.cuda.stream(self._copy_stream):
                    out = self._bufs[slot].to(self.device, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._copy_stream)
                torch.cuda.current_stream(self.device).wait_event(ev)
                out.record_stream(torch.cuda.current_stream(self.device))
                if pending is not None:
                    pending[0].synchronize()
                    self._free.put(pending[1])
                pending = (ev, slot)
            yield out
        if pending is not None:
            pending[0].synchronize()
            self._free.put(pending[1])

    def close(self):
        self._free.put(None)
        self._thread.join(timeout=10)
        if self._pool:
            lib().vo_ingest_destroy(self._pool)
            self._pool = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
