"""MI355X-native monocular VO hot path: the per-frame step and two-frame bootstrap of
ManuelWendl/Monocular_Visual_Odometry_VA4MR's VisualOdometryPipeLine as HIP kernels for gfx950
behind a C ABI (include/vo_hip.h).  Entry points: ``VisualOdometryPipeLine`` (the reference
class's surface), ``cv2compat`` (its nine cv2 calls), ``engine.Engine`` (batched chains)."""
import os as _os

# Hardware queues per process.  HIP's default of 4 lets the queue a stream lands on depend on
# the process's stream history (streams share queues round robin): a process that had captured
# one hipGraph ran the 64-shard sequence job at 25.7-25.9k instead of 29.6k frames/s; with 8
# queues the dependence is gone and every measured workload ran equal or faster
# (profiles/r4_hw_queues.txt).  HIP reads the variable when it initialises, so this takes effect
# when the package is imported before the process's first HIP call; a value already in the
# environment is kept.
_os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
