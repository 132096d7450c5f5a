/*
 * vo_hip.h -- C ABI of libvo_hip.so, the MI355X (gfx950) VO hot path.
 *
 * Drop-in boundary.  The reference has no FFI: its hot path sits behind
 * (B1) nine cv2 calls made by /root/reference/VisualOdometryPipeLine.py and (B2) the
 * VisualOdometryPipeLine class itself.  Each entry point below names the reference
 * call it replaces.  The library never allocates on a call path: every buffer is a
 * caller-owned device pointer (PyTorch tensors are used purely as containers), every
 * call is asynchronous on the given HIP stream, returns an int status (0 = OK,
 * VO_E* < 0 on bad arguments / HIP launch errors) and leaves per-chain runtime
 * outcomes (the reference's ValueError conditions) in the device status word.
 *
 * Batching: B independent VO chains ("shards") are processed per call.  State arrays
 * are [B][capacity] with per-chain device counts, so a whole per-frame step is a fixed
 * sequence of launches with no host synchronisation (hipGraph-capturable).
 */
#ifndef VO_HIP_H
#define VO_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* vo_stream_t; /* hipStream_t */

enum vo_err {
    VO_OK = 0,
    VO_EARG = -1,
    VO_EHIP = -2,
};

/* per-chain runtime status (device int32), set by the stage that detects it */
enum vo_chain_status {
    VO_ST_OK = 0,
    VO_ST_NOT_ENOUGH_KP = 1,   /* VisualOdometryPipeLine.py:357-358 ValueError      */
    VO_ST_PNP_FAILED = 2,      /* VisualOdometryPipeLine.py:351-352 ValueError      */
    VO_ST_GFTT_NONE = 3,       /* :256 goodFeaturesToTrack returned None -> crash  */
    VO_ST_GFTT_ONE = 4,        /* :256-258 single corner -> squeeze() breaks index */
    VO_ST_CAPACITY = 5,        /* a fixed capacity of this engine was exceeded     */
    VO_ST_ESSENTIAL_FAILED = 6,/* :308 findEssentialMat produced no model          */
    VO_ST_NO_MATCHES = 7,      /* :209-245 no bootstrap matches                    */
};

#define VO_MAX_LEVELS 8
#define VO_BORDER 16

/* Geometry of the per-chain image pyramid: u8 images with a VO_BORDER reflect-101 border;
 * derivative images as interleaved int16 (dx, dy) pairs with a zero border: the pixel at
 * pyramid byte offset o has dx at der[2o] and dy at der[2o + 1] (one dword per pixel).
 * The engine gives every level the pitch of level 0 (the LK kernel relies on it for
 * scalar row offsets; other pitches select the per-level LK kernels). */
typedef struct vo_dims {
    int32_t B, W, H;
    int32_t nlev;                 /* levels kept (maxLevel + 1 after the winSize cap)   */
    int32_t lvl_w[VO_MAX_LEVELS], lvl_h[VO_MAX_LEVELS], lvl_pitch[VO_MAX_LEVELS];
    int64_t lvl_off[VO_MAX_LEVELS];  /* byte offset of level l (padded origin)         */
    int64_t pyr_stride;           /* bytes per chain, u8 pyramid                          */
    int64_t der_stride;           /* int16 elements per chain (>= 2*pyr_stride): (dx, dy) */
    int32_t ncap, pcap, fcap;     /* landmark, candidate, pose capacities per chain       */
    int32_t ccap;                 /* GFTT local-maximum candidates per chain              */
    int32_t mcap;                 /* GFTT output corners per chain                        */
    int64_t work_stride;          /* fp64 scratch per chain (>= 16*max(ncap,pcap)+4096)   */
    int64_t iwork_stride;         /* int32 scratch per chain (>= 2*max(ncap,pcap)+4096)   */
} vo_dims;

/* Reference options (main.py:20-44 keys) plus host-derived constants. */
typedef struct vo_opts {
    double K[9], K_inv[9];
    double min_dist_landmarks, max_dist_landmarks;
    double min_baseline_angle;    /* degrees                                            */
    double cos_baseline;          /* smallest c with degrees(arccos(c)) < min_baseline_angle
                                     under the host's numpy (exact gate, :144-147); 2 = never */
    int32_t min_baseline_frames;
    double feature_ratio;
    int32_t feature_max_corners;
    double feature_quality_level, feature_min_dist;
    int32_t feature_block_size, feature_use_harris;
    double harris_k;
    int32_t win_w, win_h, max_level, crit_type, crit_count;
    double crit_eps;              /* raw epsilon (squared inside, as OpenCV)             */
    double min_eig;
    double pnp_conf, pnp_error;
    int32_t pnp_iters;
} vo_opts;

/* Device state of B chains; every pointer is [B][...] contiguous per chain. */
typedef struct vo_state {
    uint8_t* pyr[2];              /* ping-pong image pyramids  [B][pyr_stride]          */
    int16_t* der[2];              /* Scharr of pyr[0] / pyr[1]    [B][der_stride]       */
    float* lm_X;                  /* matched_landmarks  [B][ncap][3]                     */
    float* lm_kp;                 /* matched_keypoints  [B][ncap][2]                     */
    int32_t* nL;                  /* [B]                                                 */
    float* c_kp;                  /* potential_keys       [B][pcap][2]                   */
    float* c_first;               /* potential_first_keys [B][pcap][2]                   */
    int32_t* c_tau;               /* potential_transforms [B][pcap]                      */
    int32_t* nC;                  /* [B]                                                 */
    double* pose_R;               /* transforms (R_CW)  [B][fcap][9]                     */
    double* pose_t;               /* transforms (t_CW)  [B][fcap][3]                     */
    int32_t* nF;                  /* len(transforms) [B]                                 */
    int32_t* num_pts;             /* [B][fcap]                                           */
    float* outl_kp;               /* outlier_pts_current [B][max(ncap,pcap)][2]          */
    float* inl_kp;                /* inlier_pts_current  [B][max(ncap,pcap)][2]          */
    int32_t* nOutl;               /* [B]                                                 */
    int32_t* nInl;                /* len(inlier_pts_current) [B]                         */
    int32_t* status;              /* enum vo_chain_status [B]                            */
    /* scratch */
    float* trk_pts;               /* LK outputs [B][ncap+pcap][2]                        */
    uint8_t* trk_st;              /* LK status  [B][ncap+pcap]                           */
    float* trk_err;               /* LK err     [B][ncap+pcap]                           */
    float* eig;                   /* GFTT eigen map [B][W*H]                              */
    uint32_t* eig_max;            /* [B] order-preserving float bits                      */
    uint64_t* gf_keys;            /* [B][ccap]                                            */
    int32_t* gf_n;                /* [B]                                                  */
    float* corners;               /* [B][mcap][2]                                         */
    int32_t* nCorners;            /* [B]                                                  */
    double* pnp_rt;               /* PnP rvec,tvec [B][6]                                 */
    int32_t* pnp_ok;              /* PnP success [B]                                      */
    int32_t* pnp_ninl;            /* PnP inlier count [B]                                 */
    uint8_t* pnp_mask;            /* PnP inlier mask [B][ncap]                            */
    double* work;                 /* per-chain fp64 scratch [B][work_stride]              */
    int32_t* iwork;               /* per-chain int scratch  [B][iwork_stride]             */
    uint64_t* gf_sort;            /* GFTT selection scratch [B][ccap + VO_GF_SORT_EXTRA], zeroed
                                     at allocation (the split selection leaves it zeroed); NULL
                                     selects the one-block k_gftt_select                      */
} vo_state;

#define VO_GF_SORT_EXTRA 4096     /* u64 after the sorted keys: value histogram + counter   */

/* ---- library ---------------------------------------------------------------- */
const char* vo_version(void);
int vo_device_arch(char* buf, int len);          /* gcnArchName of the current device */
int vo_device_cus(void);                          /* compute units of the current device (or < 0) */
/* Launch-shape threshold: several entry points pick their kernel form by comparing the chain
 * count B with the device's compute units (vo_essential / vo_bootstrap / vo_triangulate /
 * vo_pnp / vo_pnp_triangulate: one block per chain at or above the CU count, split or
 * unconstrained forms below).  n > 0 makes those decisions assume n CUs (test hook: every form
 * on a small batch); n = 0 restores the device's own count.  Results never depend on it. */
int vo_set_launch_cus(int n);
/* Form of the GFTT corner selection inside vo_gftt (goodFeaturesToTrack's sort + minDistance
 * walk, VisualOdometryPipeLine.py:256): 0 = automatic (the split one-wave kernels k_gsel_* where
 * the configuration allows them, else k_gftt_select), 1 = always the one-block k_gftt_select,
 * 2 = the split form where it applies.  Test / A-B hook; the corner lists are identical. */
int vo_set_gftt_select(int mode);
/* A HIP stream of the current device whose kernels may run on every compute unit except
 * `reserve` of them (every `stride`-th CU-mask bit from stride - 1, hipExtStreamCreateWithCUMask):
 * tracking on such a stream leaves those CUs to the one-block-per-chain latency kernels of the
 * other stream groups (measurement option of the sequence job, VO_TRACK_CU_RESERVE).  The caller
 * destroys it with vo_stream_destroy. */
int vo_stream_create_cumask(int reserve, int stride, vo_stream_t* out);
int vo_stream_destroy(vo_stream_t stream);

/* ---- per-frame step stages (replace VisualOdometryPipeLine.py:326-373) --------- */

/* Build the pyramid of the new frames into state->pyr[cur] and its Scharr derivatives into
 * state->der[cur] (buildOpticalFlowPyramid + calcSharrDeriv inside cv2.calcOpticalFlowPyrLK,
 * :281,287), one fused pass per level.  frames: [B][H][W] u8, frame_stride bytes between
 * chains.  The derivative buffers' zero border is never written (allocate them zeroed). */
int vo_pyr_build(const vo_dims* d, const vo_state* s, int cur, const uint8_t* frames,
                 int64_t frame_stride, vo_stream_t stream);
/* Scharr derivatives of pyramid `which` into state->der[which] (calcSharrDeriv), border
 * included; vo_pyr_build already produces them, this recomputes them alone. */
int vo_pyr_deriv(const vo_dims* d, const vo_state* s, int which, vo_stream_t stream);

/* feature_tracking (:271-290): LK of landmarks and (if P > 1) candidates from pyr[prev]
 * to pyr[1-prev], then the reference's status filtering (ordered compaction). */
int vo_track(const vo_dims* d, const vo_opts* o, const vo_state* s, int prev, vo_stream_t stream);

/* vo_track without the filtering: the calcOpticalFlowPyrLK calls (:281, :287) into the tracking
 * scratch (trk_pts, trk_st); vo_filter_pnp_triangulate then filters (:283-290) in its PnP block. */
int vo_track_lk(const vo_dims* d, const vo_opts* o, const vo_state* s, int prev, vo_stream_t stream);

/* PnP step (:338-358): guard N >= 8, cv2.solvePnPRansac(P3P) + EPnP refit, inlier
 * filtering, Rodrigues, inversion; writes pose slot nF (not yet counted). */
int vo_pnp(const vo_dims* d, const vo_opts* o, const vo_state* s, vo_stream_t stream);

/* triangulate_landmarks (:107-206) incl. cv2.triangulatePoints per candidate (:188),
 * using pose slot nF as the current pose.  Runs only where P > 1 (:366) unless force. */
int vo_triangulate(const vo_dims* d, const vo_opts* o, const vo_state* s, int force,
                   vo_stream_t stream);

/* vo_pnp followed by vo_triangulate(force = 0) as one launch, each chain's triangulation in the
 * block that solved its pose (the engine's step; same results as the two calls).  No reference
 * counterpart of its own: it replaces the pair VisualOdometryPipeLine.py:342-358 + :366-368. */
int vo_pnp_triangulate(const vo_dims* d, const vo_opts* o, const vo_state* s, vo_stream_t stream);

/* feature_tracking's status filtering (:283-290) after vo_track_lk, then vo_pnp_triangulate, in
 * one launch (the engine's step: one kernel boundary fewer between tracking and PnP). */
int vo_filter_pnp_triangulate(const vo_dims* d, const vo_opts* o, const vo_state* s, vo_stream_t stream);

/* cv2.goodFeaturesToTrack (:256) on pyramid level 0 of pyr[cur] -> state->corners. */
int vo_gftt(const vo_dims* d, const vo_opts* o, const vo_state* s, int cur, vo_stream_t stream);

/* Diagnostics: the cornerMinEigenVal / cornerHarris map goodFeaturesToTrack thresholds
 * (featureselect.cpp), written to state->eig ([B][W*H] f32) with its max in eig_max.
 * vo_gftt itself never stores this map. */
int vo_gftt_eigmap(const vo_dims* d, const vo_opts* o, const vo_state* s, int cur, vo_stream_t stream);

/* feature_adding distance filter + append (:258-268) and the pose/num_pts append
 * (:371-373).  Call after vo_gftt. */
int vo_add_corners_finish(const vo_dims* d, const vo_opts* o, const vo_state* s, vo_stream_t stream);

/* Chain 0's (status, inlier count) written by one kernel into dst[0..1], which may be pinned host
 * memory: what the drop-in class checks after every frame to raise the reference's ValueErrors
 * (:352, :358) and to append len(inlier_pts_current) (:360-364), without a gather + copy. */
int vo_status_word(const vo_state* s, int32_t* dst, vo_stream_t stream);

/* ---- single-call primitives for the cv2 surface (B1) --------------------------- */

/* cv2.calcOpticalFlowPyrLK (:281,287): points [B][n] with per-chain counts, using the
 * pyramids/derivatives already in state (prev = pyr[prev], next = pyr[1-prev]). */
int vo_lk_points(const vo_dims* d, const vo_opts* o, const vo_state* s, int prev,
                 const float* pts, const int32_t* counts, int32_t cap, float* out_pts,
                 uint8_t* out_status, float* out_err, vo_stream_t stream);

/* cv2.solvePnPRansac(..., SOLVEPNP_P3P) (:343) on [B][cap] points with counts.
 * out: rvec[B][3], tvec[B][3], success[B], inlier mask [B][cap] (u8), n_inl[B]. */
int vo_pnp_ransac(const vo_opts* o, int B, const float* obj, const float* img,
                  const int32_t* counts, int32_t cap, double* rvec, double* tvec,
                  int32_t* success, uint8_t* inl_mask, int32_t* n_inl, double* work,
                  int64_t work_stride, vo_stream_t stream);

/* cv2.triangulatePoints (:188) for float32 points: P1,P2 [n][12] (row-major 3x4 each,
 * one pair per point), x1,x2 [n][2] -> out [n][4] float32. */
int vo_triangulate_points(int n, const double* P1, const double* P2, const float* x1,
                          const float* x2, float* out4, vo_stream_t stream);

/* cv2.Rodrigues (:354): n vectors [n][3] -> matrices [n][9], or the inverse. */
int vo_rodrigues(int n, int to_matrix, const double* in, double* out, vo_stream_t stream);

/* ---- bootstrap (initialization, :293-323) --------------------------------------- */

/* Device buffers for one SIFT invocation.  Geometry (octave sizes/offsets) is filled by
 * vo_sift_plan(); the buffers are caller-allocated with the sizes it reports. */
#define VO_SIFT_MAX_OCT 16
typedef struct vo_sift_buf {
    int32_t W, H;                 /* input image size                                   */
    int32_t n_oct;
    int32_t oct_w[VO_SIFT_MAX_OCT], oct_h[VO_SIFT_MAX_OCT];
    int64_t gauss_off[VO_SIFT_MAX_OCT * 6];   /* float offsets into gauss            */
    int64_t dog_off[VO_SIFT_MAX_OCT * 5];     /* float offsets into dog              */
    int64_t gauss_floats, dog_floats, tmp_floats;
    float* gauss;                 /* Gaussian scale space                               */
    float* dog;                   /* difference of Gaussians                            */
    float* tmp;                   /* separable-blur scratch (2W*2H floats)              */
    float* consts;                /* [7*32 kernel taps][64 exp32f table] (host-filled)  */
    int32_t* counters;            /* [8]: n_cand, n_kp, n_out, overflow, n_refined, -   */
    int32_t* cand;                /* extrema candidates [cand_cap][4] (o, layer, r, c)  */
    float* kp;                    /* raw keypoints [kp_cap][8]                          */
    float* kp_out;                /* sorted, deduplicated keypoints [kp_cap][6]         */
    float* desc;                  /* descriptors [kp_cap][128] (integer-valued floats)  */
    float* hist;                  /* descriptor histogram scratch [kp_cap][360]         */
    int32_t cand_cap, kp_cap;     /* kp_cap <= 32768 (raw keypoints sorted in LDS)       */
    int32_t nfeatures;            /* SIFT_create(nfeatures): > 0 applies retainBest      */
} vo_sift_buf;

/* Fill the geometry of `sb` for a W x H image (host only, no device work); resets
 * nfeatures to 0 (no cap). */
int vo_sift_plan(vo_sift_buf* sb, int W, int H);

/* cv2.SIFT_create().detectAndCompute(img, None) (:35,226-227) for one image;
 * sb->nfeatures > 0 is SIFT_create(nfeatures) (BASELINE C5's capped SIFT): the keypoints are
 * cut by KeyPointsFilter::retainBest in libstdc++'s nth_element/partition order. */
int vo_sift(const vo_sift_buf* sb, const uint8_t* img, int W, int H, vo_stream_t stream);

/* detectAndCompute for B images per launch sequence (the bootstrap of B chains, :226-227
 * for every chain): image b at imgs + b * img_stride; every buffer of `sb` holds B
 * consecutive per-image blocks of the size vo_sift_plan reports (gauss_floats, dog_floats,
 * tmp_floats, 8 counters, cand_cap*4, kp_cap*{8,6,128,360}).  Image b's results are bit-
 * identical to vo_sift on that image alone. */
int vo_sift_batch(const vo_sift_buf* sb, int B, const uint8_t* imgs, int64_t img_stride, int W, int H,
                  vo_stream_t stream);

/* Test hook: KeyPointsFilter::retainBest (the SIFT_create(nfeatures) cap, VisualOdometryPipeLine.py:35
 * with BASELINE C5's nfeatures) as run inside vo_sift_batch, on caller-given rows kp_out [n][6]
 * (response in column 4), reordered in place; counters[2] = n on entry, the kept count on
 * return; scratch >= 4 n + 2 ints, tmp >= 6 n floats (all device memory); n <= 32768. */
int vo_sift_retain_best_rows(float* kp_out, int32_t n, int32_t nfeatures, int32_t* counters, int32_t* scratch,
                             float* tmp, vo_stream_t stream);

/* Batched BFMatcher().knnMatch(q, t, k=2) (:36,229) for B independent problems on MFMA
 * (csrc/vo_match.hip): q [B][qcap][128], t [B][tcap][128] integer-valued float descriptors
 * (SIFT: 0..255), device counts nq[B] / nt[B]; idx2 [B][qcap][2] (-1 if absent), dist2
 * [B][qcap][2] (FLT_MAX if absent); rows >= nq[b] untouched.  Same (distance, index) order and
 * float distances as OpenCV (batchDistance + the k = 2 insertion).  scratch: device bytes >= vo_bf_knn2_batch_scratch(). */
int64_t vo_bf_knn2_batch_scratch(int B, int32_t qcap, int32_t tcap);
int vo_bf_knn2_batch(int B, const float* q, const int32_t* nq, int32_t qcap, const float* t,
                     const int32_t* nt, int32_t tcap, int32_t dim, int32_t* idx2, float* dist2,
                     void* scratch, int64_t scratch_bytes, vo_stream_t stream);

/* Ratio test + match gathering of initial_feature_matching (:218-245) for B chains:
 * keeps query i iff dist0 < ratio * dist1 (in double, as Python), in query order. */
int vo_ratio_matches(int B, const float* kp0, const float* kp1, int32_t kp_stride,
                     const int32_t* idx2, const float* dist2, const int32_t* nq, int32_t q_stride,
                     double ratio, float* pts0, float* pts1, int32_t* counts, int32_t cap,
                     vo_stream_t stream);

/* cv2.findEssentialMat(p0,p1,K,RANSAC,prob,threshold) (:308) for B problems of
 * [B][cap] points with counts; E [B][9], mask [B][cap]. */
int vo_find_essential(const vo_opts* o, int B, const float* p0, const float* p1,
                      const int32_t* counts, int32_t cap, double prob, double threshold,
                      int32_t max_iters, double* E, uint8_t* mask, int32_t* ok, double* work,
                      int32_t work_doubles, vo_stream_t stream);

/* cv2.recoverPose(E,p0,p1,K) (:315): R [B][9], t [B][3], mask [B][cap], n_good [B]. */
int vo_recover_pose(const vo_opts* o, int B, const double* E, const float* p0,
                    const float* p1, const int32_t* counts, int32_t cap, double* R, double* t,
                    uint8_t* mask, int32_t* n_good, vo_stream_t stream);

/* Bootstrap assembly into chain state (initial_feature_matching + :308-323): from the
 * per-chain bootstrap matches (pts0/pts1 [B][cap], counts) run E-RANSAC, inlier
 * filtering, recoverPose, sign fix, triangulation, pose append, num_pts. */
int vo_bootstrap(const vo_dims* d, const vo_opts* o, const vo_state* s, const float* pts0,
                 const float* pts1, const int32_t* counts, int32_t cap, vo_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif
