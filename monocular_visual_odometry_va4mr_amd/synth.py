"""Seeded synthetic monocular sequences with ground truth.

The reference reads KITTI / Malaga / Parking frames from disk (``utils.py:55-85``);
none of those datasets exist here, so every test and benchmark runs on procedurally
rendered sequences that have the reference's image sizes and intrinsics:

* KITTI 1241x376, K from ``utils.py:22-24``
* Parking 640x480, K from ``utils.py:43-45``
* Malaga 800x600 (K ``utils.py:34-36``) and 1024x768 (same K scaled by 1.28)
* 1920x1080 (KITTI focal scaled to the width)

Scene: a textured "canyon" -- ground plane, two side walls and a ceiling -- whose
texture is multi-octave value noise, band-limited per pixel by the world-space
footprint so that far surfaces fade to the mean instead of aliasing.  The camera
moves forward one unit per frame and yaws sinusoidally (bounded lateral drift).

The KITTI-size (C2) sequence uses its own scene (``PRESET_SCENES``): half a unit per
frame, seven texture octaves and no distance fading; the 1920x1080 (C5) sequence uses it too.  With the default scene the
reference orchestration loses every landmark after a few hundred frames (its monocular
scale collapses until the 1-unit minimum-depth gate rejects every triangulation,
VisualOdometryPipeLine.py:149-168); with this one it tracks all 4541 frames from frame 0
and from every 16-shard bootstrap (tools/scene_sweep.py).
Rendering is plain torch in float64 using only elementwise IEEE operations (no BLAS,
no library RNG), so a frame is bit-identical whether rendered on the CPU or the GPU
and on any host; this module is data plumbing, not part of the VO hot path.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

K_KITTI = np.array([[7.188560000000e+02, 0, 6.071928000000e+02],
                    [0, 7.188560000000e+02, 1.852157000000e+02],
                    [0, 0, 1]])                                   # utils.py:22-24
K_MALAGA = np.array([[621.18428, 0, 404.0076],
                     [0, 621.18428, 309.05989],
                     [0, 0, 1]])                                  # utils.py:34-36
K_PARKING = np.array([[331.37, 0, 320],
                      [0, 369.568, 240],
                      [0, 0, 1]])                                 # utils.py:43-45

SIZES = {
    "kitti": (1241, 376),
    "parking": (640, 480),
    "malaga": (800, 600),
    "malaga1024": (1024, 768),
    "hd1080": (1920, 1080),
}


def scene_for(preset: str) -> "SceneParams":
    return PRESET_SCENES.get(preset, SceneParams())


def intrinsics(name: str) -> np.ndarray:
    if name == "kitti":
        return K_KITTI.copy()
    if name == "parking":
        return K_PARKING.copy()
    if name == "malaga":
        return K_MALAGA.copy()
    if name == "malaga1024":
        K = K_MALAGA.copy()
        K[:2] *= 1.28
        return K
    if name == "hd1080":
        K = K_KITTI.copy()
        s = 1920.0 / 1241.0
        K[0, 0] *= s
        K[1, 1] *= s
        K[0, 2] = 959.5
        K[1, 2] = 539.5
        return K
    raise ValueError(f"unknown sequence preset {name!r}")


@dataclass
class SceneParams:
    cam_height: float = 1.65      # ground plane at y = +cam_height (y down)
    ceiling: float = 7.0          # ceiling plane at y = -ceiling
    wall: float = 9.0             # side walls at x = +-wall
    speed: float = 1.0            # units per frame along the heading
    yaw_amp_deg: float = 5.0      # heading amplitude
    yaw_period: float = 300.0     # frames per heading period
    mean: float = 110.0
    contrast: float = 90.0
    noise_sigma: float = 2.0
    octaves: int = 10
    base_wavelength: float = 8.0  # world units of the coarsest octave
    persistence: float = 1.0
    lod: bool = True              # fade octaves in with the pixel footprint (anti-aliasing)


# scene per sequence preset (default SceneParams() otherwise); see the module docstring
PRESET_SCENES = {
    "kitti": SceneParams(speed=0.5, octaves=7, lod=False),
    # C5 (BASELINE "8k keypoints/frame"): the C2 scene at 1920x1080 -- ~16k SIFT keypoints per
    # frame, so the bootstrap's SIFT_create(nfeatures=8192) cap is exercised, and a full 8,192
    # GFTT corners (the default scene gave 4.4k SIFT keypoints and ~6.5k corners)
    "hd1080": SceneParams(speed=0.5, octaves=7, lod=False),
}


def poses(n_frames: int, p: SceneParams, start: int = 0):
    """Ground-truth camera->world rotations and centres for frames [start, start+n)."""
    Rs, cs = [], []
    c = np.zeros(3)
    # integrate from frame 0 so that any window of the sequence is consistent
    for k in range(start + n_frames):
        th = math.radians(p.yaw_amp_deg) * math.sin(2.0 * math.pi * k / p.yaw_period)
        if k >= start:
            ct, st = math.cos(th), math.sin(th)
            R_wc = np.array([[ct, 0.0, st], [0.0, 1.0, 0.0], [-st, 0.0, ct]])
            Rs.append(R_wc)
            cs.append(c.copy())
        c = c + p.speed * np.array([math.sin(th), 0.0, math.cos(th)])
    return np.stack(Rs), np.stack(cs)


def _hash2(ix: torch.Tensor, iy: torch.Tensor, seed) -> torch.Tensor:
    """Integer lattice hash -> float in [-1, 1).  int64 arithmetic, identical on CPU/GPU."""
    h = ix * 374761393 + iy * 668265263 + seed * 2147483647
    h = (h ^ (h >> 13)) * 1274126177
    h = h ^ (h >> 16)
    return ((h & 0xFFFF).to(torch.float64) / 32768.0) - 1.0


def _value_noise(u: torch.Tensor, v: torch.Tensor, seed, sharp: torch.Tensor) -> torch.Tensor:
    """Lattice value noise whose cell-to-cell transition is sharpened by ``sharp``
    (1 = smooth value noise, large = anti-aliased constant tiles with corners)."""
    iu = torch.floor(u)
    iv = torch.floor(v)
    fu = ((u - iu - 0.5) * sharp + 0.5).clamp(0.0, 1.0)
    fv = ((v - iv - 0.5) * sharp + 0.5).clamp(0.0, 1.0)
    iu = iu.to(torch.int64)
    iv = iv.to(torch.int64)
    su = fu * fu * (3 - 2 * fu)
    sv = fv * fv * (3 - 2 * fv)
    n00 = _hash2(iu, iv, seed)
    n10 = _hash2(iu + 1, iv, seed)
    n01 = _hash2(iu, iv + 1, seed)
    n11 = _hash2(iu + 1, iv + 1, seed)
    a = n00 + (n10 - n00) * su
    b = n01 + (n11 - n01) * su
    return a + (b - a) * sv


class Renderer:
    """Renders frames of one seeded sequence on a torch device."""

    def __init__(self, preset: str = "kitti", seed: int = 0, device="cpu",
                 params: SceneParams | None = None):
        self.preset = preset
        self.W, self.H = SIZES[preset]
        self.K = intrinsics(preset)
        self.seed = int(seed)
        self.p = params or scene_for(preset)
        self.device = torch.device(device)
        fx, fy, cx, cy = (float(self.K[0, 0]), float(self.K[1, 1]), float(self.K[0, 2]),
                          float(self.K[1, 2]))
        ys, xs = torch.meshgrid(torch.arange(self.H, dtype=torch.float64),
                                torch.arange(self.W, dtype=torch.float64), indexing="ij")
        # camera-frame rays with elementwise IEEE ops only (bit-identical on CPU and GPU)
        self.rx = ((xs - cx) / fx).to(self.device)
        self.ry = ((ys - cy) / fy).to(self.device)
        self.inv_f = 1.0 / fx
        self.pix = (ys * self.W + xs).to(torch.int64).to(self.device)

    def gt_poses(self, n_frames: int, start: int = 0):
        return poses(n_frames, self.p, start)

    @torch.no_grad()
    def render(self, frame_idx: int, R_wc: np.ndarray, c_w: np.ndarray) -> torch.Tensor:
        return self.render_batch([frame_idx], np.asarray(R_wc)[None], np.asarray(c_w)[None])[0]

    @torch.no_grad()
    def render_batch(self, frame_idx, R_wc: np.ndarray, c_w: np.ndarray) -> torch.Tensor:
        """Render F frames at once -> uint8 [F, H, W]; per-pixel arithmetic is identical to
        rendering them one by one (every op is elementwise, per-frame scalars broadcast)."""
        p = self.p
        dev = self.device
        F = len(frame_idx)
        Rt = torch.as_tensor(np.asarray(R_wc, np.float64).reshape(F, 3, 3), device=dev)
        ct = torch.as_tensor(np.asarray(c_w, np.float64).reshape(F, 3), device=dev)
        Rk = lambda i, j: Rt[:, i, j].view(F, 1, 1)
        rx, ry = self.rx[None], self.ry[None]
        dx = rx * Rk(0, 0) + ry * Rk(0, 1) + Rk(0, 2)
        dy = rx * Rk(1, 0) + ry * Rk(1, 1) + Rk(1, 2)
        dz = rx * Rk(2, 0) + ry * Rk(2, 1) + Rk(2, 2)
        cx, cy, cz = (ct[:, i].view(F, 1, 1) for i in range(3))
        big = torch.full_like(dx, 1e9)
        eps = 1e-6
        # ground y = +h, ceiling y = -c, walls x = +-w
        t_g = torch.where(dy > eps, (p.cam_height - cy) / dy.clamp(min=eps), big)
        t_c = torch.where(dy < -eps, (-p.ceiling - cy) / dy.clamp(max=-eps), big)
        t_r = torch.where(dx > eps, (p.wall - cx) / dx.clamp(min=eps), big)
        t_l = torch.where(dx < -eps, (-p.wall - cx) / dx.clamp(max=-eps), big)
        ts = torch.stack([t_g, t_c, t_r, t_l], 0)
        del t_g, t_c, t_r, t_l, big
        t, which = ts.min(0)
        del ts
        px = cx + t * dx
        py = cy + t * dy
        pz = cz + t * dz
        # texture coordinates per surface
        u = torch.where(which < 2, px, pz)
        v = torch.where(which < 2, pz, py)
        del px, py, pz
        # pixel footprint in world units, grazing-angle aware
        dnorm = torch.sqrt(dx * dx + dy * dy + dz * dz)
        cos_inc = torch.where(which < 2, dy.abs(), dx.abs()) / dnorm
        foot = t * dnorm * self.inv_f / cos_inc.clamp(min=0.03)
        del dx, dy, dz, dnorm, cos_inc, t
        val = torch.zeros_like(u)
        amp = 1.0
        wl = p.base_wavelength
        norm = 0.0
        for o in range(p.octaves):
            att = ((wl / foot - 2.0) / 2.0).clamp(0.0, 1.0) if p.lod else 1.0
            sharp = (wl / foot / 1.5).clamp(1.0, 60.0)
            # per-surface lattice seed (seed*131 + surface*7919 + octave*31), one fused pass
            seed_t = which.to(torch.int64) * 7919 + (self.seed * 131 + o * 31)
            n = _value_noise(u / wl, v / wl, seed_t, sharp)
            val = val + amp * att * n
            norm += amp
            amp *= p.persistence
            wl *= 0.5
        img = p.mean + p.contrast * 2.0 * val / norm
        # sensor noise: Irwin-Hall(4) of hashed uniforms, exact integer hashing
        fi = torch.as_tensor([(self.seed * 1000003 + int(f)) * 2654435761 for f in frame_idx],
                             dtype=torch.int64, device=dev).view(F, 1, 1)
        base = self.pix[None] + fi
        acc = torch.zeros_like(img)
        for k in range(4):
            acc = acc + (_hash2(base, torch.full_like(base, k), 17) + 1.0) * 0.5
        noise = (acc - 2.0) * math.sqrt(3.0) * p.noise_sigma
        img = torch.round(img + noise).clamp(0, 255).to(torch.uint8)
        return img

    def frames(self, n_frames: int, start: int = 0):
        Rs, cs = self.gt_poses(n_frames, start)
        out = []
        for i in range(0, n_frames, 8):
            j = min(n_frames, i + 8)
            out.extend(self.render_batch(list(range(start + i, start + j)), Rs[i:j], cs[i:j]).unbind(0))
        return out, Rs, cs


class CachedRenderer:
    """A Renderer whose first ``n_frames`` frames are rendered once into device memory;
    ``render_batch`` then returns copies of cached frames (identical bytes: the frame index
    alone determines a frame, and the poses passed in are the sequence's own).  The bench's
    sequence legs run many slices of one sequence (~0.47 MB per KITTI frame)."""

    def __init__(self, base: Renderer, n_frames: int, chunk: int = 32):
        self.base = base
        self.preset, self.W, self.H, self.K = base.preset, base.W, base.H, base.K
        self.seed, self.p, self.device = base.seed, base.p, base.device
        Rs, cs = base.gt_poses(n_frames)
        self.cache = torch.empty((n_frames, self.H, self.W), dtype=torch.uint8, device=self.device)
        for a in range(0, n_frames, chunk):
            b = min(n_frames, a + chunk)
            self.cache[a:b] = base.render_batch(list(range(a, b)), Rs[a:b], cs[a:b])

    def gt_poses(self, n_frames: int, start: int = 0):
        return self.base.gt_poses(n_frames, start)

    @torch.no_grad()
    def render_batch(self, frame_idx, R_wc=None, c_w=None) -> torch.Tensor:
        idx = [int(i) for i in frame_idx]
        if max(idx) >= self.cache.shape[0]:
            return self.base.render_batch(frame_idx, R_wc, c_w)
        return self.cache[torch.as_tensor(idx, device=self.device)]

    def render(self, frame_idx: int, R_wc=None, c_w=None) -> torch.Tensor:
        return self.render_batch([frame_idx], R_wc, c_w)[0]


def make_sequence(preset: str, n_frames: int, seed: int = 0, start: int = 0, device="cpu"):
    """Return (frames uint8 [n,H,W] numpy, K, R_wc [n,3,3], c_w [n,3])."""
    r = Renderer(preset, seed, device)
    fr, Rs, cs = r.frames(n_frames, start)
    arr = torch.stack(fr).cpu().numpy()
    return arr, r.K, Rs, cs
