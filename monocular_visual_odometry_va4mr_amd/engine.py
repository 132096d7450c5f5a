"""Batched, device-resident VO engine: B independent chains stepped together on one GPU.

Host orchestration for the per-frame step of VisualOdometryPipeLine.continuous_operation
(/root/reference/VisualOdometryPipeLine.py:326-373).  All state lives in HBM as fixed-
capacity arrays with per-chain device counts (include/vo_hip.h ``vo_state``); a step is a
fixed sequence of C-ABI launches on one HIP stream with no host synchronisation, so it can
be captured into a hipGraph (``capture_step``).  PyTorch is used only to allocate device
memory and to obtain the current stream.

The reference's per-frame control flow maps to stages as

    feature_tracking :271-290   -> vo_pyr_build(cur) (pyramid + derivatives) + vo_track(prev)
    PnP step        :338-358    -> vo_pnp
    triangulation   :366-367    -> vo_triangulate
    feature_adding  :369        -> vo_gftt(cur) + vo_add_corners_finish (also :371-373)

(by default the filtering of feature_tracking, PnP and triangulation run as one launch:
vo_track_lk + vo_filter_pnp_triangulate; VO_PNP_TRI_SPLIT=1 selects the separate calls)

and runtime ValueErrors of the reference become per-chain status codes (``statuses``).
"""
from __future__ import annotations

import ctypes as C

import os

import numpy as np
import torch

from . import _lib as L


def pyr_max_level(w: int, h: int, win=(15, 15), max_level: int = 3) -> int:
    """Levels kept by buildOpticalFlowPyramid (stop when the next level is <= winSize)."""
    sw, sh = w, h
    for lvl in range(max_level + 1):
        sw, sh = (sw + 1) // 2, (sh + 1) // 2
        if sw <= win[0] or sh <= win[1]:
            return lvl
    return max_level


def _f64_key(x: float) -> int:
    """Order-preserving integer image of a double (for bisection over representable values)."""
    i = int(np.array([x], np.float64).view(np.int64)[0])
    return i if i >= 0 else -(i & 0x7FFFFFFFFFFFFFFF)


def _f64_from_key(k: int) -> float:
    i = k if k >= 0 else (-k) | -0x8000000000000000
    return float(np.array([i], np.int64).view(np.float64)[0])


def baseline_cos_threshold(min_angle_deg: float) -> float:
    """The baseline-angle gate of check_baseline (VisualOdometryPipeLine.py:144-147),
    ``np.degrees(np.arccos(np.clip(c, -1, 1))) < min_baseline_angle``, as a threshold on c.

    arccos is monotone, so the gate holds exactly for c >= the smallest double c* for which
    the expression is true *as this host's numpy evaluates it* (same 1-element array path as
    the reference).  The kernel then compares c >= c*, with no device acos; the two agree for
    every double c (and both are false for NaN).  Returns 2.0 when no c passes."""
    def gate(c: float) -> bool:
        return bool(np.degrees(np.arccos(np.array([c], np.float64)))[0] < min_angle_deg)
    if not gate(1.0):
        return 2.0
    if gate(-1.0):
        return -1.0
    lo, hi = _f64_key(-1.0), _f64_key(1.0)         # gate(lo) false, gate(hi) true
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if gate(_f64_from_key(mid)):
            hi = mid
        else:
            lo = mid
    return _f64_from_key(hi)


def make_opts(K: np.ndarray, options: dict) -> L.VoOpts:
    o = L.VoOpts()
    K = np.asarray(K, np.float64)
    Kinv = np.linalg.inv(K)                       # VisualOdometryPipeLine.py:38
    for i in range(9):
        o.K[i] = float(K.flat[i])
        o.K_inv[i] = float(Kinv.flat[i])
    o.min_dist_landmarks = float(options["min_dist_landmarks"])
    o.max_dist_landmarks = float(options["max_dist_landmarks"])
    o.min_baseline_angle = float(options["min_baseline_angle"])
    o.cos_baseline = baseline_cos_threshold(float(options["min_baseline_angle"]))
    o.min_baseline_frames = int(options["min_baseline_frames"])
    o.feature_ratio = float(options.get("feature_ratio", 0.8))
    o.feature_max_corners = int(options["feature_max_corners"])
    o.feature_quality_level = float(options["feature_quality_level"])
    o.feature_min_dist = float(options["feature_min_dist"])
    o.feature_block_size = int(options["feature_block_size"])
    o.feature_use_harris = int(bool(options["feature_use_harris"]))
    o.harris_k = 0.04
    o.win_w, o.win_h = (int(v) for v in options["winSize"])
    o.max_level = int(options["maxLevel"])
    ct, cc, ce = options["criteria"]
    o.crit_type, o.crit_count, o.crit_eps = int(ct), int(cc), float(ce)
    o.min_eig = 1e-4
    o.pnp_conf = float(options["PnP_conf"])
    o.pnp_error = float(options["PnP_error"])
    o.pnp_iters = int(options["PnP_iterations"])
    return o


class Engine:
    """B chains of the VO per-frame step on one device."""

    def __init__(self, K, options: dict, width: int, height: int, batch: int = 1, device=None,
                 ncap: int = 16384, pcap: int = 16384, fcap: int = 8192):
        if not torch.cuda.is_available():
            raise RuntimeError("Engine needs a ROCm GPU (no CPU fallback)")
        self.lib = L.lib()
        self.device = torch.device(device or "cuda")
        self.K = np.asarray(K, np.float64)
        self.options = dict(options)
        self.B, self.W, self.H = int(batch), int(width), int(height)
        self.opts = make_opts(self.K, options)
        d = L.VoDims()
        d.B, d.W, d.H = self.B, self.W, self.H
        win = tuple(int(v) for v in options["winSize"])
        nlev = pyr_max_level(self.W, self.H, win, int(options["maxLevel"])) + 1
        if nlev > L.VO_MAX_LEVELS:
            raise ValueError("too many pyramid levels")
        d.nlev = nlev
        off = 0
        w, h = self.W, self.H
        # one pitch for every level (that of level 0): the LK kernel addresses rows of any
        # level with scalar offsets r * pitch
        pitch = ((self.W + 2 * L.VO_BORDER + 63) // 64) * 64
        for lv in range(nlev):
            d.lvl_w[lv], d.lvl_h[lv], d.lvl_pitch[lv], d.lvl_off[lv] = w, h, pitch, off
            off += (h + 2 * L.VO_BORDER) * pitch
            w, h = (w + 1) // 2, (h + 1) // 2
        d.pyr_stride = ((off + 255) // 256) * 256 + 256   # tail slack for dword-row staging (k_lk_w)
        d.der_stride = 2 * d.pyr_stride
        d.ncap, d.pcap, d.fcap = int(ncap), int(pcap), int(fcap)
        d.ccap = self.W * self.H // 2 + 1024
        mc = int(options["feature_max_corners"])
        d.mcap = max(1, min(mc if mc > 0 else 8192, 8192))
        kmax = max(ncap, pcap)
        d.work_stride = 16 * kmax + 4096
        d.iwork_stride = 2 * kmax + 4096
        self.dims = d
        B = self.B
        dev = self.device
        z = lambda *shape, dt: torch.zeros(*shape, dtype=dt, device=dev)
        T = {}
        T["pyr0"] = z(B, d.pyr_stride, dt=torch.uint8)
        T["pyr1"] = z(B, d.pyr_stride, dt=torch.uint8)
        T["der0"] = z(B, d.der_stride, dt=torch.int16)     # (dx, dy) pairs; zero border is relied upon
        T["der1"] = z(B, d.der_stride, dt=torch.int16)
        T["lm_X"] = z(B, ncap, 3, dt=torch.float32)
        T["lm_kp"] = z(B, ncap, 2, dt=torch.float32)
        T["nL"] = z(B, dt=torch.int32)
        T["c_kp"] = z(B, pcap, 2, dt=torch.float32)
        T["c_first"] = z(B, pcap, 2, dt=torch.float32)
        T["c_tau"] = z(B, pcap, dt=torch.int32)
        T["nC"] = z(B, dt=torch.int32)
        T["pose_R"] = z(B, fcap, 9, dt=torch.float64)
        T["pose_t"] = z(B, fcap, 3, dt=torch.float64)
        T["nF"] = z(B, dt=torch.int32)
        T["num_pts"] = z(B, fcap, dt=torch.int32)
        T["outl_kp"] = z(B, kmax, 2, dt=torch.float32)
        T["inl_kp"] = z(B, kmax, 2, dt=torch.float32)
        T["nOutl"] = z(B, dt=torch.int32)
        T["nInl"] = z(B, dt=torch.int32)
        T["status"] = z(B, dt=torch.int32)
        T["trk_pts"] = z(B, ncap + pcap, 2, dt=torch.float32)
        T["trk_st"] = z(B, ncap + pcap, dt=torch.uint8)
        T["trk_err"] = z(B, ncap + pcap, dt=torch.float32)
        T["eig"] = z(B, self.W * self.H, dt=torch.float32)
        T["eig_max"] = z(B, dt=torch.int32)
        T["gf_keys"] = z(B, d.ccap, dt=torch.int64)
        T["gf_n"] = z(B, dt=torch.int32)
        T["gf_sort"] = z(B, d.ccap + L.VO_GF_SORT_EXTRA, dt=torch.int64)
        T["corners"] = z(B, d.mcap, 2, dt=torch.float32)
        T["nCorners"] = z(B, dt=torch.int32)
        T["pnp_rt"] = z(2, B, 3, dt=torch.float64)
        T["pnp_ok"] = z(B, dt=torch.int32)
        T["pnp_ninl"] = z(B, dt=torch.int32)
        T["pnp_mask"] = z(B, ncap, dt=torch.uint8)
        T["work"] = z(B, d.work_stride, dt=torch.float64)
        T["iwork"] = z(B, d.iwork_stride, dt=torch.int32)
        self.t = T
        s = L.VoState()
        for name in L._STATE_FIELDS:
            setattr(s, name, T[name].data_ptr())
        self.state = s
        self.prev = 0                      # index of the pyramid holding potential_frame
        self._pd, self._po, self._ps = C.byref(self.dims), C.byref(self.opts), C.byref(self.state)
        self._graphs = {}

    # ------------------------------------------------------------------ utils
    @property
    def stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _chk(self, rc, what):
        L.check(rc, what)

    def statuses(self) -> np.ndarray:
        return self.t["status"].cpu().numpy()

    def _sw_alloc(self):
        if getattr(self, "_sw_host", None) is None:
            self._sw_host = torch.zeros(2, dtype=torch.int32).pin_memory()

    def _sw_write(self, stream):
        """vo_status_word: chain 0's (status, inlier count) stored by one kernel straight into
        the pinned host word (mapped into the device address space)."""
        self._chk(self.lib.vo_status_word(self._ps, C.c_void_p(self._sw_host.data_ptr()), stream),
                  "vo_status_word")

    def status_word(self, in_graph: bool = False) -> tuple[int, int]:
        """(status, inlier count) of chain 0 with one host synchronisation (the drop-in class
        reads them after every frame).  ``in_graph``: the last replayed step graph already
        wrote the word."""
        self._sw_alloc()
        if not in_graph:
            self._sw_write(self.stream)
        torch.cuda.current_stream(self.device).synchronize()
        return int(self._sw_host[0]), int(self._sw_host[1])

    # ------------------------------------------------------------------ stages
    def build_pyramid(self, frames: torch.Tensor, which: int, deriv: bool = False):
        """Pyramid + Scharr derivatives of `frames` into pyr[which] / der[which] (vo_pyr_build
        always produces both; deriv=True additionally recomputes der[which] by vo_pyr_deriv)."""
        frames = self._frames(frames)
        self._drain_prefetch()
        self._chk(self.lib.vo_pyr_build(self._pd, self._ps, which, C.c_void_p(frames.data_ptr()),
                                        self.W * self.H, self.stream), "vo_pyr_build")
        if deriv:
            self._chk(self.lib.vo_pyr_deriv(self._pd, self._ps, which, self.stream), "vo_pyr_deriv")

    def _drain_prefetch(self):
        """Order a pending next-frames pyramid build (step(next_frames=...)) before whatever the
        caller launches next on the current stream, and drop it: only step() itself may consume
        it (graph replays, captures and explicit pyramid builds write the same
        pyramid buffers)."""
        pre, self._pre = getattr(self, "_pre", None), None
        if pre is not None:
            torch.cuda.current_stream(self.device).wait_event(pre[0])

    def _frames(self, frames):
        if not isinstance(frames, torch.Tensor):
            frames = torch.as_tensor(np.ascontiguousarray(frames))
        if frames.dim() == 2:
            frames = frames.unsqueeze(0)
        if frames.dtype != torch.uint8 or tuple(frames.shape) != (self.B, self.H, self.W):
            raise ValueError(f"frames must be uint8 [{self.B},{self.H},{self.W}]")
        return frames.to(self.device, non_blocking=True).contiguous()

    STAGES = ("pyr_build", "track", "pnp", "triangulate", "gftt", "add_finish")

    def step(self, frames, marks=None, next_frames=None):
        """One continuous_operation for every chain (frames: uint8 [B,H,W], any device).

        ``marks``: optional callable ``marks(stage_index, end, stream)`` invoked on the
        launching thread right before (end=False) and after (end=True) each stage, with
        the torch stream that stage runs on (bench.py records HIP events there).

        ``next_frames``: the following step's frames when they are already known (a sequence
        in memory).  Their pyramid is then built during this step -- on the side stream, as
        soon as this step's tracking (the last reader of that pyramid buffer) is issued -- and
        the next step, given the same frames, starts with tracking.  Same kernels, same bytes;
        the drop-in class, fed one frame per call, never passes it.  The prefetch is queued on
        the side stream behind this step's GFTT.  Used up to 16 chains per engine, where GFTT
        ends early (rank 0 of the 8-GPU sequence plan, 2 x 12 chains: 83.2-84.4k -> 88.2-89.7k
        frames/s predicted), and from 256 chains, where the split GFTT selection (round 6) ends
        well inside the step's tracking (headline 67.9-68.7k -> 69.7-70.0k frames/s,
        profiles/r6/prefetch_ab.jsonl).  At 24 chains GFTT ends after the next step would have
        started (48-chain sequence 36.9k -> 34.7k, also in round 6); C5's 128 chains per engine
        are neutral.  VO_PREFETCH=0 / 1 forces it off / on."""
        frames = self._frames(frames)
        nxt = None
        mode = os.environ.get("VO_PREFETCH", "")
        if next_frames is not None and (mode == "1" or (mode != "0" and (self.B <= 16 or self.B >= 256))):
            nxt = self._frames(next_frames)
        self._step_launch(frames, self.prev, marks, nxt=nxt)
        self.prev = 1 - self.prev

    def _side_stream(self):
        if os.environ.get("VO_ONE_STREAM") == "1":      # profiling: every stage on the main stream
            return torch.cuda.current_stream(self.device)
        if getattr(self, "_side", None) is None:
            # Streams share the process's few hardware queues round-robin, so a pool stream can
            # land on the main stream's queue, which serialises GFTT behind PnP (one chain in a
            # process that had made other streams: 0.75 instead of 0.50 ms per frame).  For
            # small batches the side stream comes from the high-priority pool, whose queues are
            # never those of a normal-priority main stream.
            hi = self.B <= 16 or self._prio_latency()
            self._side = torch.cuda.Stream(self.device, priority=-1 if hi else 0)
        return self._side

    @staticmethod
    def _prio_latency() -> bool:
        return os.environ.get("VO_PRIO_LATENCY") == "1"

    def _latency_stream(self):
        """VO_PRIO_LATENCY=1: the one-block-per-chain stages (PnP + triangulation, the step
        finish) on a high-priority stream of their own, so that the dispatcher hands them CUs
        before the queued tracking blocks of another stream group (measurement option)."""
        if getattr(self, "_lat", None) is None:
            self._lat = torch.cuda.Stream(self.device, priority=-1)
        return self._lat

    def _step_launch(self, frames, prev, marks=None, gftt_late=False, nxt=None):
        """Stage DAG of one step on two streams.  main: pyramid + Scharr derivatives of the
        new frame (pyr[cur], der[cur]) -> track(prev) -> PnP + triangulate -> [join] ->
        add_finish.  side: GFTT on the new frame (needs only its pyramid,
        VisualOdometryPipeLine.py:253), overlapping tracking and PnP.  GFTT never writes the
        chain status (PnP owns it while the two run; see k_gftt_select).
        ``gftt_late``: issue GFTT after tracking (same DAG).  A captured graph then runs the
        tracking branch on the pyramid's queue and GFTT, which has slack, across queues:
        one chain replays ~17 us faster (GFTT first made tracking wait ~33 us for the
        cross-queue dependency); eager launches keep the plain order."""
        cur = 1 - prev
        lib = self.lib
        main = torch.cuda.current_stream(self.device)
        side = self._side_stream()
        sm, ss = C.c_void_p(main.cuda_stream), C.c_void_p(side.cuda_stream)
        pd, po, ps = self._pd, self._po, self._ps
        fp = C.c_void_p(frames.data_ptr())
        names = self.STAGES

        def run(i, strm, call):
            if marks is not None:
                marks(i, False, strm)
            self._chk(call(), "vo_" + names[i])
            if marks is not None:
                marks(i, True, strm)

        forked = side.cuda_stream != main.cuda_stream
        # pyramid(cur) built during the previous step (next_frames) for these very frames
        pre, self._pre = getattr(self, "_pre", None), None
        if pre is not None:
            main.wait_event(pre[0])                               # the prefetch wrote pyr[cur]
        if pre is not None and forked and pre[1] == (frames.data_ptr(), frames._version, cur) and not gftt_late:
            run(0, main, lambda: 0)
        else:
            run(0, main, lambda: lib.vo_pyr_build(pd, ps, cur, fp, self.W * self.H, sm))
        if forked:
            side.wait_stream(main)                                # pyramid(cur) ready, last step's corners consumed
        if not gftt_late:
            run(4, side, lambda: lib.vo_gftt(pd, po, ps, cur, ss))
        fused = getattr(self, "fuse_pnp_tri", os.environ.get("VO_PNP_TRI_SPLIT") != "1")
        # fused: tracking leaves the status filtering (:283-290) to the PnP launch, which runs it
        # first in each chain's block (one kernel boundary fewer on the step's critical path)
        defer = fused and os.environ.get("VO_COMPACT_IN_TRACK") != "1"      # =1: A/B option
        track = lib.vo_track_lk if defer else lib.vo_track
        ts = getattr(self, "track_stream", None)
        if ts is not None and forked and not gftt_late:
            # tracking on a stream shared by the engines of a batch (track_stream): their LK
            # launches run one after another instead of side by side, so one group's PnP,
            # feature adding and next pyramid overlap the other group's tracking
            ts.wait_stream(main)                                  # pyramid(cur) built
            run(1, ts, lambda: track(pd, po, ps, prev, C.c_void_p(ts.cuda_stream)))
            main.wait_stream(ts)
        else:
            run(1, main, lambda: track(pd, po, ps, prev, sm))
        if gftt_late:
            run(4, side, lambda: lib.vo_gftt(pd, po, ps, cur, ss))
        ev_corners = None
        if forked:
            ev_corners = torch.cuda.Event()
            ev_corners.record(side)                               # corners ready (before any prefetch)
        if nxt is not None and forked and not gftt_late:
            # the next frames' pyramid into pyr[prev] / der[prev], which this step's tracking
            # (just issued on main) is the last to read.  (On a stream of its own instead of
            # behind this step's GFTT it was slower: the streams share four hardware queues.)
            pst = side
            pst.wait_stream(main)
            nxt.record_stream(pst)                                # keep the frames alive for that stream
            # marked as this step's stage 0 (the build it replaces is the next step's, which
            # then records an empty stage 0): the per-stage report keeps one build per step
            if marks is not None:
                marks(0, False, pst)
            self._chk(lib.vo_pyr_build(pd, ps, prev, C.c_void_p(nxt.data_ptr()), self.W * self.H,
                                       C.c_void_p(pst.cuda_stream)), "vo_pyr_build")
            if marks is not None:
                marks(0, True, pst)
            ev_pre = torch.cuda.Event()
            ev_pre.record(pst)
            self._pre = (ev_pre, (nxt.data_ptr(), nxt._version, prev))
        lat = main
        if self._prio_latency() and forked:
            lat = self._latency_stream()
            lat.wait_stream(main)                                 # tracking done
        sl = C.c_void_p(lat.cuda_stream)
        if fused:
            # one launch for filtering, PnP and triangulation (vo_filter_pnp_triangulate); stage 3
            # is then empty
            pnp = lib.vo_filter_pnp_triangulate if defer else lib.vo_pnp_triangulate
            run(2, lat, lambda: pnp(pd, po, ps, sl))
            run(3, lat, lambda: 0)
        else:
            run(2, lat, lambda: lib.vo_pnp(pd, po, ps, sl))
            run(3, lat, lambda: lib.vo_triangulate(pd, po, ps, 0, sl))
        if forked:
            lat.wait_event(ev_corners)                            # corners ready
        run(5, lat, lambda: lib.vo_add_corners_finish(pd, po, ps, sl))
        if lat is not main:
            main.wait_stream(lat)                                 # the step ends on main

    def capture_step(self):
        """Capture the two ping-pong variants of the step into hipGraphs; returns the device
        frame buffer bound at capture time (step_graph copies each frame there).  Measured on
        one chain (tools/graph_probe.py), the replay is not faster than eager launches, which
        overlap the GPU anyway: the drop-in class steps eagerly by default.  A frames pointer
        read by the kernels from a pinned host slot instead of the copy cost ~60 us per frame
        (system-scope reads of host memory) and was dropped (round 6)."""
        self._drain_prefetch()
        torch.cuda.synchronize(self.device)            # nothing pending crosses into the capture
        buf = torch.zeros((self.B, self.H, self.W), dtype=torch.uint8, device=self.device)
        self._sw_alloc()
        graphs = []
        side = torch.cuda.Stream(self.device)
        for prev in (0, 1):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(side):
                with torch.cuda.graph(g, stream=side):
                    self._step_launch(buf, prev, gftt_late=True)
                    # the status word of chain 0 as the graph's last node, written into pinned
                    # host memory (status_word then only waits)
                    self._sw_write(C.c_void_p(side.cuda_stream))
            graphs.append(g)
        torch.cuda.synchronize(self.device)
        self._graphs = {"buf": buf, "g": graphs}
        return buf

    def replay_step(self):
        self._drain_prefetch()
        g = self._graphs["g"][self.prev]
        g.replay()
        self.prev = 1 - self.prev

    def step_graph(self, frames):
        """Same as step(), replayed from a captured hipGraph (one launch per frame; the frames
        are copied into the graph's bound buffer first: host frames directly, device frames by
        one device copy)."""
        if not self._graphs:
            self.capture_step()
        buf = self._graphs["buf"]
        if not isinstance(frames, torch.Tensor):
            frames = torch.as_tensor(np.ascontiguousarray(frames))
        if frames.dim() == 2:
            frames = frames.unsqueeze(0)
        if frames.dtype != torch.uint8 or tuple(frames.shape) != tuple(buf.shape):
            raise ValueError(f"frames must be uint8 [{self.B},{self.H},{self.W}]")
        buf.copy_(frames)
        self.replay_step()

    # ------------------------------------------------------------------ bootstrap
    def reserve_bootstrap(self, sift_batch_bytes: int | None = None):
        """Allocate the SIFT scale-space workspace bootstrap() uses (SIFT_create at
        VisualOdometryPipeLine.py:35 is likewise done once, in the constructor); bootstrap()
        calls it itself when nothing is reserved.  Returns (Sift, chains per chunk)."""
        from .features import Sift
        budget = int(sift_batch_bytes or os.environ.get("VO_SIFT_BATCH_BYTES", 64 << 30))
        per_img = Sift.bytes_per_image(self.W, self.H)
        m = max(1, min(self.B, budget // (2 * per_img)))     # chains per chunk
        nfeat = int(self.options.get("sift_nfeatures", 0))    # C5: SIFT_create(8192)
        if getattr(self, "_sift", None) is None or self._sift.batch < 2 * m or self._sift.nfeatures != nfeat:
            self._sift = None
            torch.cuda.empty_cache()
            self._sift = Sift(self.W, self.H, self.device, batch=2 * m, nfeatures=nfeat)
            self._load_bootstrap_glue()
        return self._sift, m

    def _load_bootstrap_glue(self):
        """Run the bootstrap's few torch-side glue ops (strided counter reads, the capacity-flag
        merge, the status select) once on the fresh workspace's zeroed counters, so that their
        GPU code is loaded here, with the workspace, and not in the first bootstrap: HIP loads a
        kernel's code object at its first launch, and one such load inside the first bootstrap
        blocked the host for 0.1 s (GPU idle up to 44 ms, tools/boot_api_trace.sh).  Writes
        nothing the bootstrap reads (the results are discarded)."""
        c = self._sift.t["counters"][:2]
        f = c[:, 3]
        ovf = torch.zeros(1, dtype=torch.int32, device=self.device)
        ovf[0:1] = torch.maximum(f[:1], f[1:])
        n = c[:, 2].contiguous()
        ovf[0:1] = n[:1]
        torch.where(ovf > 0, torch.full_like(ovf, L.ST_CAPACITY), ovf)

    def release_bootstrap(self):
        """Free the SIFT workspace and the matcher scratch (stepping never needs them)."""
        self._sift = None
        self._mscr = None
        torch.cuda.empty_cache()

    def bootstrap(self, img0, img1, sift_batch_bytes: int | None = None):
        """initialization (VisualOdometryPipeLine.py:293-323) for every chain on the GPU:
        SIFT on both frames, BF 2-NN + ratio test, 5-point E-RANSAC, inlier split,
        recoverPose, t *= sign(t_z), triangulation, pose append; then potential_frame
        = img1 (its pyramid + derivatives become pyr[prev]).  Option ``sift_nfeatures`` (the C5
        preset's 8192) is SIFT_create(nfeatures).

        Batched across chains: the chains are taken in chunks whose SIFT scale spaces fit
        ``sift_batch_bytes`` (default 64 GB, env VO_SIFT_BATCH_BYTES); per chunk one
        vo_sift_batch over both frames of every chain, one vo_bf_knn2_batch over its pairs
        and one vo_ratio_matches; then one vo_bootstrap for all chains.  No host sync: a chain
        whose SIFT keypoints hit the capacity ends with status VO_ST_CAPACITY."""
        self._drain_prefetch()
        from .features import bf_knn2_batch, matcher_scratch_bytes
        img0 = self._frames(img0)
        img1 = self._frames(img1)
        d = self.dims
        dev = self.device
        B = self.B
        # a workspace the caller reserved stays (reserve_bootstrap / release_bootstrap); one
        # allocated here is freed at the end, so stepping never holds up to the SIFT budget
        own = getattr(self, "_sift", None) is None
        sift, m = self.reserve_bootstrap(sift_batch_bytes)
        kcap = sift.kp_cap
        cap = min(d.ncap, d.pcap, kcap)
        pts0 = torch.zeros((B, cap, 2), dtype=torch.float32, device=dev)
        pts1 = torch.zeros_like(pts0)
        cnt = torch.zeros(B, dtype=torch.int32, device=dev)
        n0 = torch.zeros(B, dtype=torch.int32, device=dev)
        n1 = torch.zeros_like(n0)
        ovf = torch.zeros(B, dtype=torch.int32, device=dev)      # per chain: SIFT capacity hit
        st = self.stream
        # the matcher's scratch belongs to this engine: engines bootstrapping on
        # their own streams never share one, and no allocation happens inside the chunk loop
        mbytes = max(matcher_scratch_bytes(min(B, c0 + m) - c0, kcap, kcap) for c0 in {0, (B - 1) // m * m})
        if getattr(self, "_mscr", None) is None or self._mscr.numel() < mbytes:
            self._mscr = torch.empty(mbytes, dtype=torch.uint8, device=dev)
        for c0 in range(0, B, m):
            c1 = min(B, c0 + m)
            k = c1 - c0
            kp, desc, n = sift.run_batch(torch.cat([img0[c0:c1], img1[c0:c1]]))
            flag = sift.t["counters"][:2 * k, 3]
            ovf[c0:c1] = torch.maximum(flag[:k], flag[k:])
            n0[c0:c1] = n[:k]
            n1[c0:c1] = n[k:]
            idx2, dist2 = bf_knn2_batch(desc[:k], n[:k], desc[k:], n[k:], scratch=self._mscr)
            self._chk(self.lib.vo_ratio_matches(k, C.c_void_p(kp[:k].data_ptr()), C.c_void_p(kp[k:].data_ptr()), kcap,
                                                C.c_void_p(idx2.data_ptr()), C.c_void_p(dist2.data_ptr()),
                                                C.c_void_p(n[:k].data_ptr()), kcap, float(self.opts.feature_ratio),
                                                C.c_void_p(pts0[c0:c1].data_ptr()), C.c_void_p(pts1[c0:c1].data_ptr()),
                                                C.c_void_p(cnt[c0:c1].data_ptr()), cap, st), "vo_ratio_matches")
        self._chk(self.lib.vo_bootstrap(self._pd, self._po, self._ps, C.c_void_p(pts0.data_ptr()),
                                        C.c_void_p(pts1.data_ptr()), C.c_void_p(cnt.data_ptr()), cap, st),
                  "vo_bootstrap")
        # a chain whose keypoint set was truncated by the SIFT capacity must not run on: its status
        # becomes VO_ST_CAPACITY on the device (every stage skips it, statuses() / the drop-in
        # class report it) -- no host synchronisation inside the bootstrap
        self.t["status"].copy_(torch.where(ovf > 0, torch.full_like(ovf, L.ST_CAPACITY), self.t["status"]))
        self.prev = 0
        self.build_pyramid(img1, self.prev)
        self._boot_debug = {"n0": n0, "n1": n1, "pts0": pts0, "pts1": pts1, "cnt": cnt}
        if own:
            # the caching allocator only reuses the blocks once the queued kernels are done
            # with them; dropping the references is stream-ordered, so no synchronisation
            self._sift = None
            self._mscr = None

    # ------------------------------------------------------------------ state I/O
    def import_chain(self, b: int, *, landmarks, keypoints, cand, cand_first, cand_tau, transforms,
                     num_pts, prev_img):
        """Load reference-shaped state into chain b (checkpoint restore / test hook)."""
        d = self.dims
        T = self.t
        lm = np.asarray(landmarks, np.float32).reshape(-1, 3)
        kp = np.asarray(keypoints, np.float32).reshape(-1, 2)
        c = np.asarray(cand, np.float32).reshape(-1, 2)
        cf = np.asarray(cand_first, np.float32).reshape(-1, 2)
        ct = np.asarray(cand_tau).reshape(-1).astype(np.int32)
        if lm.shape[0] > d.ncap or c.shape[0] > d.pcap or len(transforms) >= d.fcap:
            raise ValueError("state exceeds engine capacity")
        dev = self.device
        T["lm_X"][b, :lm.shape[0]] = torch.from_numpy(lm).to(dev)
        T["lm_kp"][b, :kp.shape[0]] = torch.from_numpy(kp).to(dev)
        T["nL"][b] = lm.shape[0]
        T["c_kp"][b, :c.shape[0]] = torch.from_numpy(c).to(dev)
        T["c_first"][b, :cf.shape[0]] = torch.from_numpy(cf).to(dev)
        T["c_tau"][b, :ct.shape[0]] = torch.from_numpy(ct).to(dev)
        T["nC"][b] = c.shape[0]
        Rs = np.stack([np.asarray(R, np.float64).reshape(9) for R, _ in transforms])
        ts = np.stack([np.asarray(t, np.float64).reshape(3) for _, t in transforms])
        T["pose_R"][b, :len(transforms)] = torch.from_numpy(Rs).to(dev)
        T["pose_t"][b, :len(transforms)] = torch.from_numpy(ts).to(dev)
        T["nF"][b] = len(transforms)
        npts = np.asarray(num_pts, np.int32).reshape(-1)
        if npts.size:
            T["num_pts"][b, 1:1 + npts.size] = torch.from_numpy(npts).to(dev)
        T["status"][b] = 0
        img = torch.as_tensor(np.ascontiguousarray(prev_img, np.uint8)).to(dev)
        # rebuild the potential_frame pyramid + derivatives for this chain only
        full = torch.zeros((self.B, self.H, self.W), dtype=torch.uint8, device=dev)
        full[b] = img
        keep = T["pyr%d" % self.prev].clone(), T["der%d" % self.prev].clone()
        self.build_pyramid(full, self.prev)
        mask = torch.zeros(self.B, dtype=torch.bool, device=dev)
        mask[b] = True
        T["pyr%d" % self.prev][~mask] = keep[0][~mask]
        T["der%d" % self.prev][~mask] = keep[1][~mask]

    def export_chain(self, b: int) -> dict:
        T = self.t
        torch.cuda.synchronize(self.device)
        nL, nC, nF = int(T["nL"][b]), int(T["nC"][b]), int(T["nF"][b])
        nI, nO = int(T["nInl"][b]), int(T["nOutl"][b])
        R = T["pose_R"][b, :nF].cpu().numpy().reshape(-1, 3, 3)
        t = T["pose_t"][b, :nF].cpu().numpy().reshape(-1, 3, 1)
        return {
            "landmarks": T["lm_X"][b, :nL].cpu().numpy(),
            "keypoints": T["lm_kp"][b, :nL].cpu().numpy(),
            "cand": T["c_kp"][b, :nC].cpu().numpy(),
            "cand_first": T["c_first"][b, :nC].cpu().numpy(),
            "cand_tau": T["c_tau"][b, :nC].cpu().numpy().astype(np.float64).reshape(-1, 1),
            "transforms": [(R[i], t[i]) for i in range(nF)],
            "num_pts": T["num_pts"][b, 1:nF].cpu().numpy(),
            "inliers": T["inl_kp"][b, :nI].cpu().numpy(),
            "outliers": T["outl_kp"][b, :nO].cpu().numpy(),
            "status": int(T["status"][b]),
        }

    def pyramid_level(self, which: int, level: int, b: int = 0) -> np.ndarray:
        d = self.dims
        w, h, p, o = d.lvl_w[level], d.lvl_h[level], d.lvl_pitch[level], d.lvl_off[level]
        buf = self.t["pyr%d" % which][b, o:o + (h + 2 * L.VO_BORDER) * p].view(h + 2 * L.VO_BORDER, p)
        return buf[L.VO_BORDER:L.VO_BORDER + h, L.VO_BORDER:L.VO_BORDER + w].cpu().numpy()

    def deriv_level(self, level: int, b: int = 0, which: int | None = None) -> np.ndarray:
        """Scharr (dx, dy) of pyramid `which` (default: the potential_frame's, pyr[prev])."""
        d = self.dims
        which = self.prev if which is None else which
        w, h, p, o = d.lvl_w[level], d.lvl_h[level], d.lvl_pitch[level], d.lvl_off[level]
        n = (h + 2 * L.VO_BORDER) * p
        # interleaved (dx, dy) int16 pairs: the pixel at pyramid byte offset o is der[2o], der[2o + 1]
        buf = self.t["der%d" % which][b].view(-1, 2)[o:o + n].view(h + 2 * L.VO_BORDER, p, 2)
        return buf[L.VO_BORDER:L.VO_BORDER + h, L.VO_BORDER:L.VO_BORDER + w].cpu().numpy()
