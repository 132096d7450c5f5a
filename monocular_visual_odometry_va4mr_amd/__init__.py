"""MI355X-native monocular VO hot path: the per-frame step and two-frame bootstrap of
ManuelWendl/Monocular_Visual_Odometry_VA4MR's VisualOdometryPipeLine as HIP kernels for gfx950
behind a C ABI (include/vo_hip.h).  Entry points: ``VisualOdometryPipeLine`` (the reference
class's surface), ``cv2compat`` (its nine cv2 calls), ``engine.Engine`` (batched chains)."""
# Hardware queues per process: the package leaves GPU_MAX_HW_QUEUES alone (importing it
# used to set 8).  Every launch-shape and stream threshold was measured on the GPU box, whose
# environment exports HIP's default of 4, and at the round-6 headline 8 queues were not faster
# (68.3k / 67.7k vs 68.8k / 68.8k frames/s alternating, profiles/r6/hwq_groups_ab.jsonl);
# bench.py --hw-queues N sets it for experiments.
