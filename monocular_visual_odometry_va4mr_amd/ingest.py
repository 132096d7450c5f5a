"""Frame ingest: dataset images -> pinned host batches -> HBM.

The reference reads one frame per step with cv2.imread(path, IMREAD_GRAYSCALE)
(utils.py:55-81).  Here libvo_ingest.so decodes a whole batch of PNGs (KITTI, Parking; one
frame per chain) on a pool of host threads into pinned memory, a Python thread keeps one
batch ahead of the consumer, and the host->HBM copy runs on its own stream, so decoding and
the copy overlap the GPU step of the previous batch.

Malaga's JPEGs go through libjpeg (via PIL, which releases the GIL while decoding) on a
thread pool, asking the decoder for grayscale output the way OpenCV's JPEG reader does for
IMREAD_GRAYSCALE (out_color_space = JCS_GRAYSCALE: the Y channel, no RGB round trip).
rocJPEG is not part of this ROCm image, so there is no device JPEG path.  Parity with
OpenCV's bundled libjpeg-turbo is unpinned (no cv2 here); both use the ISLOW IDCT.
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


_PNG_SIG = b"\x89PNG\r\n\x1a\n"
_JPEG_SIG = b"\xff\xd8\xff"


def is_jpeg(path: str) -> bool:
    with open(path, "rb") as f:
        return f.read(3) == _JPEG_SIG


def jpeg_gray(path: str, out: np.ndarray | None = None) -> np.ndarray:
    """Y channel of a baseline/progressive JPEG as uint8 [H, W] (libjpeg grayscale output)."""
    from PIL import Image
    with Image.open(path) as im:
        if im.format != "JPEG":
            raise ValueError(f"{path}: not a JPEG")
        im.draft("L", im.size)              # decoder-side colour conversion to gray, scale 1/1
        if im.mode != "L":                  # CMYK / odd layouts: fall back to PIL's conversion
            im = im.convert("L")
        arr = np.asarray(im, dtype=np.uint8)
    if out is None:
        return arr.copy()
    if out.shape != arr.shape:
        raise ValueError(f"{path}: size {arr.shape[::-1]} != expected {out.shape[::-1]}")
    out[...] = arr
    return out


def imread_gray(path: str) -> np.ndarray:
    """cv2.imread(path, cv2.IMREAD_GRAYSCALE) for the datasets' PNG and JPEG files
    (utils.py:59,70,81)."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:3] == _JPEG_SIG:
        return jpeg_gray(path)
    w, h, _, _ = png_info(data)
    out = np.empty((h, w), np.uint8)
    rc = lib().vo_png_decode_gray(data, len(data), out.ctypes.data, w, w, h)
    if rc:
        raise ValueError(f"{path}: PNG decode failed (code {rc})")
    return out


class FrameSource:
    """Iterate over batches of PNG/JPEG paths (batches[j][b] = frame of chain b at step j) and yield
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
        self._threads = int(threads)
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
            jpg = [i for i, p in enumerate(paths) if p.lower().endswith((".jpg", ".jpeg"))]
            st = np.zeros(len(paths), np.int32)
            rc = 0
            if len(jpg) < len(paths):
                png = [i for i in range(len(paths)) if i not in set(jpg)] if jpg else list(range(len(paths)))
                if len(png) == len(paths):
                    arr = (C.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
                    rc = L.vo_ingest_png_files(self._pool, arr, len(paths), self._bufs[slot].data_ptr(),
                                               self.H * self.W, self.W, self.H, st.ctypes.data)
                else:                       # mixed batch: PNGs one by one through the pool
                    for i in png:
                        arr = (C.c_char_p * 1)(os.fsencode(paths[i]))
                        one = np.zeros(1, np.int32)
                        r = L.vo_ingest_png_files(self._pool, arr, 1, self._bufs[slot][i].data_ptr(),
                                                  self.H * self.W, self.W, self.H, one.ctypes.data)
                        st[i] = one[0]
                        rc = rc or r
            if jpg:
                host = self._bufs[slot].numpy()

                def dec(i):
                    try:
                        jpeg_gray(paths[i], host[i])
                        return 0
                    except Exception:       # reported below like a PNG decode failure
                        return -4
                for i, r in zip(jpg, self._jpeg_pool().map(dec, jpg)):
                    st[i] = r
                    rc = rc or r
            self._ready.put((j, slot, rc, st))
        self._ready.put(None)

    def _jpeg_pool(self):
        if getattr(self, "_jpool", None) is None:
            from concurrent.futures import ThreadPoolExecutor
            self._jpool = ThreadPoolExecutor(max_workers=self._threads)
        return self._jpool

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
        if getattr(self, "_jpool", None) is not None:
            self._jpool.shutdown(wait=True)
            self._jpool = None
        if self._pool:
            lib().vo_ingest_destroy(self._pool)
            self._pool = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
