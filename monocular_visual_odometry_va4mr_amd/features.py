"""Device-side SIFT and brute-force matching used by the bootstrap (VisualOdometryPipeLine.py
:209-245): ``cv2.SIFT_create().detectAndCompute`` and ``cv2.BFMatcher().knnMatch(k=2)``
run by libvo_hip.so (csrc/vo_sift.hip).  Buffers are allocated once per image size."""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib as L


def default_kp_cap(width: int, height: int) -> int:
    """Raw keypoints held per image (sorted in LDS: at most 32,768): 16,384 up to a megapixel,
    32,768 above (the dense C5 1920x1080 scene yields ~16k keypoints after deduplication)."""
    return 16384 if int(width) * int(height) <= (1 << 20) else 32768


class Sift:
    """SIFT for one image size on one device (OpenCV 4.6 defaults; ``nfeatures`` > 0 is
    SIFT_create(nfeatures), BASELINE C5's capped SIFT), ``batch`` images per launch sequence
    (vo_sift_batch).  Buffers hold ``batch`` per-image blocks: results of image b are
    kp_out[b], desc[b], counters[b, 2]."""

    def __init__(self, width: int, height: int, device=None, cand_cap: int = 131072, kp_cap: int | None = None,
                 batch: int = 1, nfeatures: int = 0):
        if kp_cap is None:
            kp_cap = default_kp_cap(width, height)
        self.lib = L.lib()
        self.device = torch.device(device or "cuda")
        self.W, self.H = int(width), int(height)
        self.batch = int(batch)
        sb = L.VoSiftBuf()
        L.check(self.lib.vo_sift_plan(C.byref(sb), self.W, self.H), "vo_sift_plan")
        dev = self.device
        n = self.batch
        self.t = {
            "gauss": torch.empty(n * sb.gauss_floats, dtype=torch.float32, device=dev),
            "dog": torch.empty(n * sb.dog_floats, dtype=torch.float32, device=dev),
            "tmp": torch.empty(n * sb.tmp_floats, dtype=torch.float32, device=dev),
            "consts": torch.zeros(7 * 32 + 64, dtype=torch.float32, device=dev),
            "counters": torch.zeros(n, 8, dtype=torch.int32, device=dev),
            "cand": torch.empty(n * cand_cap * 4, dtype=torch.int32, device=dev),
            "kp": torch.empty(n * kp_cap * 8, dtype=torch.float32, device=dev),
            "kp_out": torch.zeros(n, kp_cap, 6, dtype=torch.float32, device=dev),
            "desc": torch.zeros(n, kp_cap, 128, dtype=torch.float32, device=dev),
            "hist": torch.empty(n * kp_cap * 360, dtype=torch.float32, device=dev),
        }
        for k, v in self.t.items():
            setattr(sb, k, v.data_ptr())
        sb.cand_cap, sb.kp_cap = int(cand_cap), int(kp_cap)
        sb.nfeatures = int(nfeatures)
        self.nfeatures = int(nfeatures)
        self.sb = sb
        self.kp_cap = int(kp_cap)

    @staticmethod
    def bytes_per_image(width: int, height: int, cand_cap: int = 131072, kp_cap: int | None = None) -> int:
        if kp_cap is None:
            kp_cap = default_kp_cap(width, height)
        sb = L.VoSiftBuf()
        L.check(L.lib().vo_sift_plan(C.byref(sb), int(width), int(height)), "vo_sift_plan")
        return 4 * (sb.gauss_floats + sb.dog_floats + sb.tmp_floats + 8 + cand_cap * 4 + kp_cap * (8 + 6 + 128 + 360))

    def run_batch(self, imgs: torch.Tensor):
        """Detect + describe imgs uint8 [n, H, W] (n <= batch, device-resident, contiguous);
        returns views kp_out [n, kp_cap, 6], desc [n, kp_cap, 128] and a contiguous copy of
        the keypoint counts int32 [n] (all stream-ordered, no host sync)."""
        if imgs.dtype != torch.uint8 or imgs.dim() != 3 or tuple(imgs.shape[1:]) != (self.H, self.W):
            raise ValueError("SIFT input must be uint8 [n, H, W]")
        n = int(imgs.shape[0])
        if not 1 <= n <= self.batch:
            raise ValueError(f"at most {self.batch} images per call")
        imgs = imgs.to(self.device).contiguous()
        st = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        L.check(self.lib.vo_sift_batch(C.byref(self.sb), n, C.c_void_p(imgs.data_ptr()), self.W * self.H,
                                       self.W, self.H, st), "vo_sift_batch")
        self._img = imgs      # keep alive until the stream consumes it
        return self.t["kp_out"][:n], self.t["desc"][:n], self.t["counters"][:n, 2].contiguous()

    def run(self, img: torch.Tensor):
        """Detect + describe one image; results stay on the device (kp_out, desc, count)."""
        if img.dtype != torch.uint8 or tuple(img.shape) != (self.H, self.W):
            raise ValueError("SIFT input must be uint8 [H, W]")
        k, d, n = self.run_batch(img.reshape(1, self.H, self.W))
        return k[0], d[0], n

    def overflowed(self, n: int | None = None) -> bool:
        c = self.t["counters"][: (n or 1), 3]
        return bool(int(c.max()))

    def result(self, b: int = 0):
        n = int(self.t["counters"][b, 2])
        if int(self.t["counters"][b, 3]):
            raise RuntimeError("SIFT capacity exceeded (raise cand_cap / kp_cap)")
        return self.t["kp_out"][b, :n].cpu().numpy(), self.t["desc"][b, :n].cpu().numpy()


_SCRATCH: dict = {}


def _scratch(dev, nbytes: int) -> torch.Tensor:
    """Matcher scratch per (device, stream), grown on demand (kept so repeated calls do not
    allocate).  Per stream: engines bootstrapping concurrently on streams of their own (the
    sequence job's stream groups, the headline's two engines) must not share it -- one shared
    buffer per device let one group's match overwrite the other's staged rows (found in round 4
    when the groups' bootstraps overlapped more: half the shards of one group differed from the
    reference runs)."""
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    buf = _SCRATCH.pop(key, None)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(int(nbytes), dtype=torch.uint8, device=dev)
    _SCRATCH[key] = buf                    # most recently used last
    # streams come and go (every sequence run makes its own): keep the 8 most recent buffers.
    # A dropped buffer was allocated on its own stream, so the caching allocator hands its
    # memory only to later work of that stream, after the work already queued there.
    while len(_SCRATCH) > 8:
        _SCRATCH.pop(next(iter(_SCRATCH)))
    return buf


def matcher_scratch_bytes(B: int, qcap: int, tcap: int) -> int:
    """Device bytes bf_knn2_batch needs for B problems of qcap x tcap descriptors."""
    n = int(L.lib().vo_bf_knn2_batch_scratch(int(B), int(qcap), int(tcap)))
    if n <= 0:
        raise ValueError("bad matcher sizes")
    return n


def bf_knn2_batch(q: torch.Tensor, nq: torch.Tensor, t: torch.Tensor, nt: torch.Tensor,
                  scratch: torch.Tensor | None = None):
    """k=2 nearest neighbours for B problems on MFMA (vo_bf_knn2_batch).
    q [B,qcap,128] / t [B,tcap,128] float32 integer-valued descriptors, nq / nt int32 [B] device
    counts; returns idx2 [B,qcap,2] i32 (-1 absent), dist2 [B,qcap,2] f32 (FLT_MAX absent).
    ``scratch``: a uint8 device buffer the caller owns and uses only on this stream (an Engine
    keeps one; ``matcher_scratch_bytes`` sizes it); None takes the per-stream cache."""
    if q.dim() != 3 or t.dim() != 3 or q.shape[2] != 128 or t.shape[2] != 128 or q.shape[0] != t.shape[0]:
        raise ValueError("q, t must be float32 [B, cap, 128] with the same B")
    dev = q.device
    B, qcap, tcap = int(q.shape[0]), int(q.shape[1]), int(t.shape[1])
    q = q.contiguous()
    t = t.contiguous()
    # every entry is written by the call (absent pairs as -1 / FLT_MAX)
    idx2 = torch.empty((B, qcap, 2), dtype=torch.int32, device=dev)
    dist2 = torch.empty((B, qcap, 2), dtype=torch.float32, device=dev)
    lib = L.lib()
    nbytes = int(lib.vo_bf_knn2_batch_scratch(B, qcap, tcap))
    if nbytes <= 0:
        raise ValueError("bad matcher sizes")
    if scratch is not None:
        if scratch.dtype != torch.uint8 or scratch.device != dev or scratch.numel() < nbytes:
            raise ValueError(f"matcher scratch must be uint8 on {dev} with >= {nbytes} bytes")
        scr = scratch
    else:
        scr = _scratch(dev, nbytes)
    st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    L.check(lib.vo_bf_knn2_batch(B, C.c_void_p(q.data_ptr()), C.c_void_p(nq.data_ptr()), qcap,
                                 C.c_void_p(t.data_ptr()), C.c_void_p(nt.data_ptr()), tcap, 128,
                                 C.c_void_p(idx2.data_ptr()), C.c_void_p(dist2.data_ptr()),
                                 C.c_void_p(scr.data_ptr()), nbytes, st), "vo_bf_knn2_batch")
    return idx2, dist2


def bf_knn2(q: torch.Tensor, nq: torch.Tensor, t: torch.Tensor, nt: torch.Tensor, qcap: int):
    """k=2 nearest neighbours of one problem (device counts), returns idx2 [qcap,2] i32,
    dist2 [qcap,2] f32: the batched MFMA matcher with B = 1."""
    q = q[:qcap]
    i2, d2 = bf_knn2_batch(q[None], nq.reshape(1), t[None], nt.reshape(1))
    return i2[0], d2[0]
