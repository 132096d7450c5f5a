"""Drop-in replacement for the reference ``VisualOdometryPipeLine`` class (boundary B2).

Same constructor, methods and public attributes as
/root/reference/VisualOdometryPipeLine.py:4-373, as read by the reference driver
(main.py:118-124, :170-195):

    VisualOdometryPipeLine(K, options)
    .initialization(img0, img1)          -> :293-323 (SIFT, BF ratio test, E-RANSAC, ...)
    .continuous_operation(img)           -> :326-373 (KLT, PnP-RANSAC, triangulation, GFTT)
    .transforms, .num_pts, .matched_landmarks, .matched_keypoints, .potential_keys,
    .potential_first_keys, .potential_transforms, .inlier_pts_current,
    .outlier_pts_current, .num_tracked_landmarks_list, .potential_frame, .K, .K_inv

The whole hot path runs on the GPU through libvo_hip.so (engine.Engine with one chain);
state stays in HBM and the attributes are read back on access.  The per-frame step is
launched stage by stage (asynchronous launches overlap the GPU); ``use_graph=True`` captures
it once into a pair of hipGraphs (ping-pong pyramids) and replays them,
identical results but not faster on one chain (tools/graph_probe.py: 0.45-0.51 vs 0.44-0.46 ms
per frame), so eager is the default.  The reference's failure
conditions raise the same exceptions: ValueError("Not enough keypoints for PnP") (:358),
ValueError("PnP failed") (:352), and the crashes the reference would hit when
goodFeaturesToTrack yields 0 / 1 corners (:256-258).
"""
from __future__ import annotations

import numpy as np

from . import _lib as L
from .engine import Engine


class VisualOdometryPipeLine:
    def __init__(self, K, options, max_frames: int = 8192, landmark_capacity: int = 16384,
                 candidate_capacity: int = 16384, device=None, use_graph: bool = False):
        self.options = options
        self.K = K
        self.K_inv = np.linalg.inv(K)
        self.matched_descriptors = []                  # never written by the reference (Q6)
        self.num_tracked_landmarks_list = []
        self._caps = (int(landmark_capacity), int(candidate_capacity), int(max_frames))
        self._device = device
        self._use_graph = bool(use_graph)     # per-frame step replayed from a captured hipGraph
        self._eng: Engine | None = None
        self._frame = None
        self._boot_done = False

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _as_frame(img):
        """numpy image (as the reference passes, utils.py:55-81) or a uint8 torch tensor
        already on the device (no host round trip)."""
        import torch
        return img if isinstance(img, torch.Tensor) else np.asarray(img)

    def _engine_for(self, img):
        h, w = tuple(img.shape[:2])
        if self._eng is None or (self._eng.W, self._eng.H) != (w, h):
            nc, pc, fc = self._caps
            self._eng = Engine(self.K, self.options, w, h, batch=1, device=self._device, ncap=nc, pcap=pc, fcap=fc)
        return self._eng

    def _raise_status(self, st: int):
        if st == L.ST_OK:
            return
        if st == L.ST_NOT_ENOUGH_KP:
            raise ValueError("Not enough keypoints for PnP")
        if st == L.ST_PNP_FAILED:
            raise ValueError("PnP failed")
        if st == L.ST_GFTT_NONE:
            raise AttributeError("'NoneType' object has no attribute 'squeeze'")
        if st == L.ST_GFTT_ONE:
            raise IndexError("too many indices for array: array is 1-dimensional, but 2 were indexed")
        raise RuntimeError(L.STATUS_NAMES.get(st, f"chain status {st}"))

    def _status(self) -> int:
        return int(self._eng.t["status"][0])

    # ------------------------------------------------------------------ API
    def initialization(self, img0, img1):
        img0, img1 = self._as_frame(img0), self._as_frame(img1)
        eng = self._engine_for(img1)
        eng.bootstrap(img0[None], img1[None])
        self._frame = img1
        self._boot_done = True
        self._raise_status(self._status())

    def continuous_operation(self, img):
        if not self._boot_done:
            raise RuntimeError("initialization() must run first")
        eng = self._eng
        img = self._as_frame(img)
        if self._use_graph:
            eng.step_graph(img[None])
        else:
            eng.step(img[None])
        self._frame = img
        st, n_inl = eng.status_word(in_graph=self._use_graph)  # one host sync per frame
        # the reference appends to the ring (:360-364) after PnP succeeded and before
        # feature_adding (:369), so a frame that then crashes in goodFeaturesToTrack (:256)
        # has already appended its inlier count
        if st in (L.ST_OK, L.ST_GFTT_NONE, L.ST_GFTT_ONE):
            if len(self.num_tracked_landmarks_list) == 20:
                self.num_tracked_landmarks_list.pop(0)
            self.num_tracked_landmarks_list.append(n_inl)
        self._raise_status(st)

    # ------------------------------------------------------------------ attributes
    def _field(self, name, n_name, shape_tail):
        if self._eng is None:
            return []
        n = int(self._eng.t[n_name][0])
        return self._eng.t[name][0, :n].cpu().numpy().reshape((n,) + shape_tail)

    @property
    def transforms(self):
        if self._eng is None:
            return [(np.eye(3), np.zeros((3, 1)))]
        nF = int(self._eng.t["nF"][0])
        R = self._eng.t["pose_R"][0, :nF].cpu().numpy().reshape(-1, 3, 3)
        t = self._eng.t["pose_t"][0, :nF].cpu().numpy().reshape(-1, 3, 1)
        return [(R[i], t[i]) for i in range(nF)]

    @property
    def num_pts(self):
        if self._eng is None:
            return []
        nF = int(self._eng.t["nF"][0])
        return [int(v) for v in self._eng.t["num_pts"][0, 1:nF].cpu().numpy()]

    @property
    def matched_landmarks(self):
        return self._field("lm_X", "nL", (3,))

    @property
    def matched_keypoints(self):
        return self._field("lm_kp", "nL", (2,))

    @property
    def potential_keys(self):
        return self._field("c_kp", "nC", (2,))

    @property
    def potential_first_keys(self):
        return self._field("c_first", "nC", (2,))

    @property
    def potential_transforms(self):
        if self._eng is None:
            return []
        n = int(self._eng.t["nC"][0])
        return self._eng.t["c_tau"][0, :n].cpu().numpy().astype(np.float64).reshape(n, 1)

    @property
    def inlier_pts_current(self):
        return None if not self._boot_done else self._field("inl_kp", "nInl", (2,))

    @property
    def outlier_pts_current(self):
        return None if not self._boot_done else self._field("outl_kp", "nOutl", (2,))

    @property
    def potential_frame(self):
        return self._frame

    @property
    def potential_descriptors(self):
        """Dead state in the reference (Q6: stops being filtered, never read); not kept."""
        return np.zeros((0, 128), np.float32)
