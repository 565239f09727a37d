/*
 * slam_hip.h -- C-ABI of libslam_hip.so, the MI355X (gfx950) implementation of
 * the per-step SLAM state-estimation hot path of takuyani/SLAM-Robot_Simu.
 *
 * The reference is pure Python/NumPy with no FFI of its own; these entry points
 * are what a ctypes binding of its estimator classes binds.
 * Every function below names the reference interface it replaces.
 *
 * Conventions
 *   - Plain pointers and sizes only.  Host buffers are caller-owned and are only
 *     read/written during the call; device memory is owned by the handle.
 *   - Return 0 on success, a negative SLAM_ERR_* code on failure;
 *     slam_last_error() (thread-local) describes the last failure.
 *   - A handle is not thread-safe (the reference is single-threaded).
 *   - All arithmetic is IEEE fp64, as in the reference.
 */
#ifndef SLAM_HIP_H
#define SLAM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SLAM_OK 0
#define SLAM_ERR_ARG (-1)
#define SLAM_ERR_HIP (-2)
/* particle_filter.py:219: a resample position beyond the last cumulative
 * weight raises IndexError in the reference; the device clamps to NP-1 and
 * reports this code from the call that hit it. */
#define SLAM_ERR_INDEX (-3)
#define SLAM_ERR_STATE (-4)
/* slam_graph_optimize: the PCG solve of an iteration did not converge within
 * pcg_max_iter (the dense path's singular gate is not an error: is_calc = 0
 * ends the loop as in graph_based_slam.py:706-709). */
#define SLAM_ERR_SOLVE (-5)
#define SLAM_ERR_COMM (-6)

int slam_version(void);
const char* slam_last_error(void);
int slam_device_count(int* n);

/* ====================================================================
 * Particle filter -- replaces ParticleFilter (particle_filter.py:18-237)
 * ==================================================================== */
typedef struct slam_pf slam_pf;

enum { SLAM_MOTION_LINEAR = 0,     /* particle_filter.py:121-142 (x' = A x + B u) + N(0,Q) */
       SLAM_MOTION_VELOCITY = 1 }; /* motion_model.py:31-62 (sample_motion_model_velocity) */
enum { SLAM_LIK_PRODUCT = 0,       /* particle_filter.py:185-192: sequential product of NL densities */
       SLAM_LIK_LOGSUM = 1 };      /* same density as exp(-sum(q)/2) * den^-NL (one exp per particle) */

typedef struct {
    double dt;            /* particle_filter.py:30  DT_s = period_ms / 1000 */
    double ess_threshold; /* particle_filter.py:33  ESS_TH = NP / 100 */
    double r_cov[4];      /* particle_filter.py:68-70 R (2x2, row-major) */
    double q_factor[9];   /* device-RNG noise map: noise_j = sum_k g_k q_factor[3k+j]
                             (numpy: sqrt(s)[:,None]*v of svd(Q), particle_filter.py:165) */
    double alphas[6];     /* motion_model.py:20-29 a1..a6 (velocity motion model) */
    double x0[3];         /* particle_filter.py:74-81 initial pose of every particle */
    uint64_t seed;        /* device RNG (Philox-4x32-10) key */
    int32_t motion;       /* SLAM_MOTION_* */
    int32_t likelihood;   /* SLAM_LIK_* */
} slam_pf_config;

typedef struct {
    double x_est[3];      /* particle_filter.py:117  px[:, argmax] */
    double cov[9];        /* weighted particle covariance (np.cov(px, aweights=pw, bias=True)) */
    double max_val;       /* particle_filter.py:115 */
    double ess;           /* 1 / sum(w^2) of the normalised weights after this step */
    double weight_sum;    /* particle_filter.py:234 np.sum before normalisation */
    int64_t max_idx;      /* particle_filter.py:116 (first index on ties) */
    int32_t resampled;    /* this step ran the resampling branch (particle_filter.py:211) */
    int32_t resample_next;/* ess < ESS_TH: the next step will resample */
    int32_t status;       /* bit0: resample clamp (reference IndexError); bit1: exact-scan fallback */
    int32_t n_special;    /* exact-cumsum diagnostics: sequentially folded elements */
    int32_t ess_near;     /* |ess - ESS_TH| <= band * ESS_TH: the reference's `1 / (pw @ pw.T)`
                             (particle_filter.py:210, BLAS order) could decide resample_next
                             differently; the drop-in confirms such steps on the host */
    int32_t dd_waves;     /* closed-form log-sum: wavefronts that took the double-double form
                             (a sharded step's result: the first held shard's count only) */
} slam_pf_result;

/* ParticleFilter.__init__ (particle_filter.py:21-84).  landmarks: n_landmarks x 2 row-major. */
int slam_pf_create(const slam_pf_config* cfg, int64_t n_particles, int32_t n_landmarks,
                   const double* landmarks, int device, slam_pf** out);
int slam_pf_destroy(slam_pf* h);
int slam_pf_set_landmarks(slam_pf* h, const double* landmarks);
/* Any pointer may be NULL (left unchanged).  Arrays of NP doubles. */
int slam_pf_set_state(slam_pf* h, const double* x, const double* y, const double* th,
                      const double* w);
int slam_pf_get_state(slam_pf* h, double* x, double* y, double* th, double* w);
/* The last step's weights before normalisation (w_un = pw * bn, particle_filter.py:194)
 * and the divisor the device formed for them (np.sum(w_un) in numpy's order,
 * :234; = slam_pf_result.weight_sum of that step; 1 after set_state / resample).
 * The current weights are w_un / s (:235, NaN -> 1/NP).  Either pointer may be
 * NULL.  Lets a caller pin the step-end np.sum and the reductions against
 * numpy on the device's own w_un.  Single-GPU (deferred) handles. */
int slam_pf_get_weights_raw(slam_pf* h, double* w_un, double* s);

/* One estimator step of main_pf (particle_filter.py:102-117):
 * resampling (if the previous step's ESS < ESS_TH) -> predict -> likelihood ->
 * normalise -> estimate.
 *   control:  (v, omega)                         (particle_filter.py:46-58)
 *   z:        NL x 2 robot-frame observations    (particle_filter.py:151-153)
 *   noise:    NP x 3 host array or NULL.  LINEAR: additive (x, y, yaw) noise =
 *             np.random.multivariate_normal(0, Q, NP) (particle_filter.py:165);
 *             VELOCITY: standard normals in draw order (v, w, gamma) per particle
 *             (motion_model.py:46-48).  NULL: on-device Philox stream.
 *   u_resample: rand() of particle_filter.py:214 (ofs = u / NP); NaN: device RNG. */
int slam_pf_step(slam_pf* h, const double* control, const double* z, const double* noise,
                 double u_resample, slam_pf_result* res);

/* Stage entry points (the reference's private methods). */
int slam_pf_resample(slam_pf* h, double u_resample, int32_t force, int32_t* resampled);  /* __resampling :200-224 */
int slam_pf_predict(slam_pf* h, const double* control, const double* noise);            /* __predict :156-168 */
int slam_pf_update(slam_pf* h, const double* z, slam_pf_result* res);                    /* __likelihood + estimate :113-117 */
/* Exact systematic-resampling indices for the CURRENT weights (idx_out: NP int64). */
int slam_pf_resample_indices(slam_pf* h, double u_resample, int64_t* idx_out, int32_t* n_special);
/* numpy-order np.sum of the current weights (particle_filter.py:234). */
int slam_pf_weight_sum(slam_pf* h, double* sum_out);
/* Diagnostics: the device RNG's six standard normals of particle pairs
 * [p0, p0 + count) at RNG step rstep (the perf-mode motion noise, Philox-4x32-10
 * / Philox-2x32-10 + Box-Muller; not a reference interface), out: count x 6. */
int slam_debug_pair_normals(int device, uint64_t p0, int64_t count, uint32_t rstep, uint64_t seed,
                            double* out);

/* Device-resident multi-step run (bench path): observations for n_steps steps
 * are uploaded once; steps are enqueued back to back with no host sync.  A
 * run is one setup launch (controls read from pinned host memory, counters,
 * the first step's closed-form words unless the previous run's last step
 * formed them for the same control), the steps' graphs (1/2/4/8-step shapes,
 * binary decomposition of n_steps), and one wait: the last step's finalize
 * stores the batch's result records into pinned host memory itself. */
int slam_pf_load_observations(slam_pf* h, int32_t n_steps, const double* z_all);
int slam_pf_run(slam_pf* h, int32_t first_step, int32_t n_steps, const double* controls,
                slam_pf_result* results);

/* Kernel timing (HIP events on the handle's stream; disables step graphs).
 * kernel: 0 = fused resample-gather+predict+likelihood, 1 = np.sum order
 * sums + normalise + reductions, 2 = exact-cumsum passes, 3 = whole step. */
int slam_pf_enable_timing(slam_pf* h, int32_t on);
int slam_pf_timing(slam_pf* h, int32_t kernel, double* total_ms, int64_t* launches);
/* slam_pf_run replays one captured hipGraph per step (default on). */
int slam_pf_set_graphs(slam_pf* h, int32_t on);
/* Capture every graph slam_pf_run will replay (1-, 2-, 4- and 8-step graphs for
 * both ping-pong parities) without running them, so that no capture lands in
 * a timed run; *capture_ms (may be NULL) = host time spent.  Graphs are
 * dropped (and captured again on demand) by the calls that change a step's
 * launches (set_stream, set_scan_merged, set_ess_band, the device stream). */
int slam_pf_prepare_graphs(slam_pf* h, double* capture_ms);
/* Exact cumsum of a resample step in one launch (on = default where the grid
 * is co-resident; SLAM_ERR_ARG elsewhere) or in two; bit-identical results. */
int slam_pf_set_scan_merged(slam_pf* h, int32_t on);
/* Overrides the resample decision of the next step (particle_filter.py:210-211,
 * `ess < ESS_TH`): the caller re-forms ESS as the reference does, `1 / (pw @ pw.T)`
 * on the host's BLAS, when the device's ESS lies within rounding of the
 * threshold (the device sums in its own fixed order).  Single-GPU handles. */
int slam_pf_set_resample_next(slam_pf* h, int32_t on);
/* Band of slam_pf_result.ess_near, relative to ESS_TH (default 1e-9): the steps
 * whose device ESS lies this close to the threshold, where the reference's BLAS
 * dot (particle_filter.py:210) could order the sum differently. */
int slam_pf_set_ess_band(slam_pf* h, double band);
/* external != 0: run on the caller's HIP stream (e.g. torch.cuda.current_stream();
 * NULL = the default stream).  external == 0: a private stream again. */
int slam_pf_set_stream(slam_pf* h, void* hip_stream, int32_t external);

/* ====================================================================
 * MotionModel -- replaces motion_model.py:14-86 for a batch of poses
 * (batch = 1 is the reference's single call).
 *   params:  dt, a1..a6                                   (motion_model.py:20-29)
 *   poses:   n x 3 (x, y, theta) host array; out: n x 3 (may alias poses)
 *   normals: n x 3 standard normals, per pose in the draw order (v, w, gamma)
 *            of moveWithNoise (:46-48; the std handed to normal() is sigma**2,
 *            kept); NULL: moveWithoutNoise (:64-86).
 * ==================================================================== */
int slam_motion_velocity(const double* params, int64_t n, const double* poses, double v, double w,
                         const double* normals, double* out, int device);

/* ====================================================================
 * RCCL communicator (one process per GPU).  RCCL is loaded at run time
 * (dlopen librccl.so.1); slam_comm_unique_id on one rank, the 128 bytes
 * broadcast by the caller's bootstrap, slam_comm_create on every rank.
 * ==================================================================== */
typedef struct slam_comm slam_comm;
int slam_comm_unique_id(uint8_t* id_out /* 128 bytes */);
int slam_comm_create(const uint8_t* id, int32_t world, int32_t rank, int device, slam_comm** out);
int slam_comm_destroy(slam_comm* comm);
int slam_comm_info(slam_comm* comm, int32_t* world, int32_t* rank);
/* recv (host, world * bytes) <- send (host, bytes) of every rank (bootstrap data) */
int slam_comm_all_gather_host(slam_comm* comm, const void* send, void* recv, int64_t bytes);

/* ====================================================================
 * Sharded particle filter, device-resident step (BASELINE config 3).
 * One filter of n_global particles split into contiguous shards; a
 * slam_dist groups the shards this process holds -- all of them (LOCAL:
 * several shards on one GPU, phases enqueued shard by shard on one stream) or
 * one (one process per GPU).  Exchanges are peer-memory pushes into every
 * rank's exchange region (fine-grained HBM, opened by the peers through IPC
 * handles) with device-side signalling; every kernel gates on the device
 * resample flag, so a step needs no host decision and slam_dist_run replays
 * K steps per hipGraph.  Results are identical on every rank and bit-identical
 * to one handle holding all particles (particle_filter.py:102-117).
 * ==================================================================== */
typedef struct slam_dist slam_dist;
/* the standard split: rank r holds [gbase, gbase + n_local) */
int slam_dist_shard_range(int64_t n_global, int32_t world, int32_t rank, int64_t* gbase,
                          int64_t* n_local);
/* a shard handle for slam_dist (device RNG; every shard but the last holds a
 * multiple of 8192 particles) */
int slam_pf_create_dist_shard(const slam_pf_config* cfg, int64_t n_local, int64_t n_global,
                              int64_t gbase, int32_t n_landmarks, const double* landmarks, int device,
                              slam_pf** out);
/* shards: the held shards in rank order (n_held == world: LOCAL, ranks 0..world-1;
 * n_held == 1: rank rank0, connect before stepping).  The shards must outlive it. */
int slam_dist_create(slam_pf** shards, int32_t n_held, int32_t world, int32_t rank0, slam_dist** out);
int slam_dist_destroy(slam_dist* d);
/* bootstrap blob per rank: the exchange region's IPC handle and the GPU's PCI bus id */
int slam_dist_handle_size(int64_t* bytes);
int slam_dist_export(slam_dist* d, void* blob);                 /* n_held x handle size */
/* world x handle size, rank order.  Preflight: every peer GPU must be visible and
 * reachable (hipDeviceCanAccessPeer), else SLAM_ERR_COMM before any IPC mapping. */
int slam_dist_connect(slam_dist* d, const void* all_blobs);
int slam_dist_connect_comm(slam_dist* d, slam_comm* comm);      /* export + RCCL all-gather + connect */
/* Collective exchange instead of the peer-memory stores (the fallback when a peer's
 * region cannot be mapped; replaces connect): every step's record all-gather
 * (particle_filter.py:234 normalisation across shards: the ranks' np.sum buffer
 * partials gathered, then folded in rank order on every rank -- bit-identical to
 * one GPU) and, on resample steps, the specials' and items' exchanges as RCCL
 * all-gathers and grouped send/recv between the step's kernels.  comm: an RCCL
 * communicator of the filter's world (one held shard, rank = comm rank); NULL with
 * every shard held (LOCAL), the collectives then being device copies.  Steps are
 * host-orchestrated (no hipGraphs; the host reads the resample flag each step and
 * the exchanged counts on resample steps). */
int slam_dist_set_collective(slam_dist* d, slam_comm* comm);
/* one step from host inputs (observations staged in slot 0, device RNG) */
int slam_dist_step(slam_dist* d, const double* control, const double* z, slam_pf_result* res);
/* Every wait on a peer is bounded (~2^24 polls); one that expires returns
 * SLAM_ERR_COMM and marks the handle dead: every later step or run of it fails
 * at once with SLAM_ERR_COMM (the shards' exchange state is no longer
 * consistent).  Recover by destroying and recreating every shard and the
 * slam_dist on every rank. */
int slam_dist_load_observations(slam_dist* d, int32_t n_steps, const double* z_all);
int slam_dist_run(slam_dist* d, int32_t first_step, int32_t n_steps, const double* controls,
                  slam_pf_result* results);
/* slam_pf_prepare_graphs for the sharded step (after connect) */
int slam_dist_prepare_graphs(slam_dist* d, double* capture_ms);
/* resample exchange form: 1 = one launch (the default with one held shard whose
 * scan grid is co-resident), 0 = five launches; on < 0 only reports */
int slam_dist_set_merged(slam_dist* d, int32_t on, int32_t* active);

/* ====================================================================
 * EKF localisation -- replaces ExtendedKalmanFilter
 * (extended_kalman_filter.py:17-205) for a batch of independent filters
 * (batch = 1 is the reference's single filter).  State on the device is
 * structure-of-arrays: x[3][batch], P[9][batch] (row-major 3x3).
 * ==================================================================== */
typedef struct slam_ekf slam_ekf;

typedef struct {
    double dt;            /* extended_kalman_filter.py:29  DT_s */
    double vel;           /* :46-48  V (control, also in jacobF :188) */
    double omega;         /* :46     omega */
    double q[9];          /* :62-66  Q (process noise, 3x3) */
    double r[4];          /* :68-70  R (observation noise, 2x2) */
    double x0[3];         /* :74-79  initial estimate */
    double p0[9];         /* :81-84  initial covariance */
    int32_t motion;       /* SLAM_MOTION_LINEAR: the reference's __f / jacobF / Q (:160-194);
                             SLAM_MOTION_VELOCITY: prediction driven by motion_model.py --
                             f = moveWithoutNoise (:64-86), its Jacobian G, and
                             Q = V M V^T from a1..a6 (M = diag(sv^4, sw^4): the std handed
                             to np.random.normal is sigma**2, :43-48) + the gamma yaw term */
    int32_t pad0;
    double alphas[6];     /* motion_model.py:20-29 a1..a6 (VELOCITY) */
} slam_ekf_config;

/* ExtendedKalmanFilter.__init__: every filter starts at (x0, p0). */
int slam_ekf_create(const slam_ekf_config* cfg, int64_t batch, int device, slam_ekf** out);
int slam_ekf_destroy(slam_ekf* h);
int slam_ekf_set_state(slam_ekf* h, const double* x /* batch x 3 */, const double* P /* batch x 9 */);
int slam_ekf_get_state(slam_ekf* h, double* x /* batch x 3 */, double* P /* batch x 9 */);
/* The filter half of main_ekf (extended_kalman_filter.py:108-128): prediction
 * with jacobF, Kalman gain with inv(S), update, limit_angle on the yaw,
 * P = (I - G C) P_m.  control = {v, omega} or NULL for the configured values;
 * z: batch x 2 world positions (:141-146).  Outputs may be NULL. */
int slam_ekf_step(slam_ekf* h, const double* control, const double* z, double* x_hat_m,
                  double* x_hat, double* P);
/* n_steps filter steps in one launch (state stays in registers):
 * z_all: n_steps x batch x 2; x_hat_all: n_steps x batch x 3 or NULL;
 * the final state is kept in the handle. */
int slam_ekf_run(slam_ekf* h, int32_t n_steps, const double* control, const double* z_all,
                 double* x_hat_all);
/* Device-resident variant (bench path): z_dev / x_hat_dev are device pointers
 * (x_hat_dev may be NULL); asynchronous on the handle's stream. */
int slam_ekf_run_device(slam_ekf* h, int32_t n_steps, const double* control, const double* z_dev,
                        double* x_hat_dev);
/* Bench path without foreign device buffers: upload n_steps x batch x 2
 * observations once, then run them from HBM (asynchronous; the estimates of
 * every step are kept on the device when keep_history != 0). */
int slam_ekf_load_observations(slam_ekf* h, int32_t n_steps, const double* z_all);
int slam_ekf_run_loaded(slam_ekf* h, int32_t n_steps, const double* control, int32_t keep_history);
int slam_ekf_synchronize(slam_ekf* h);

/* ====================================================================
 * EKF-SLAM (BASELINE config 4, an extension: the reference has no EKF-SLAM).
 * State mu = (robot x, y, yaw, landmark_0 x, y, phi, ...), n = 3 + 3 * n_lm;
 * P is n x n fp64 in HBM (7.2 GB at n = 30,003).  Robot motion is the
 * reference EKF's model (extended_kalman_filter.py:160-194); the landmark
 * measurement is graph_based_slam.py's ScanSensor (range, bearing,
 * orientation; :150-153) with its covariance (:187-194).
 * ==================================================================== */
typedef struct slam_ekfslam slam_ekfslam;

typedef struct {
    double dt;            /* motion step (s) */
    double q_robot[9];    /* robot process noise */
    double r_dist;        /* ScanSensor range noise fraction  (graph_based_slam.py:187-192) */
    double r_dir;         /* bearing noise (rad) */
    double r_orient;      /* orientation noise (rad) */
    int32_t motion;       /* robot motion: SLAM_MOTION_LINEAR (+ q_robot) or SLAM_MOTION_VELOCITY
                             (motion_model.py, as slam_ekf_config.motion; q_robot unused) */
    int32_t pad0;
    double alphas[6];     /* motion_model.py a1..a6 (VELOCITY) */
} slam_ekfslam_config;

int slam_ekfslam_create(const slam_ekfslam_config* cfg, int64_t n_landmarks, int device,
                        slam_ekfslam** out);
int slam_ekfslam_destroy(slam_ekfslam* h);
/* mu: n; P: n x n row-major (only the lower triangle is read). */
int slam_ekfslam_set_state(slam_ekfslam* h, const double* mu, const double* P);
/* mu: n; P <- diag(p_diag) (n values) without an n x n host buffer. */
int slam_ekfslam_init_diag(slam_ekfslam* h, const double* mu, const double* p_diag);
/* P may be NULL; when given it receives the full symmetric n x n matrix. */
int slam_ekfslam_get_state(slam_ekfslam* h, double* mu, double* P);
/* k rows of the symmetric P (rows[k] indices; out: k x n), O(k n) -- for
 * checking a 7.2 GB P without copying it to the host. */
int slam_ekfslam_get_rows(slam_ekfslam* h, int64_t k, const int64_t* rows, double* out);
/* Prediction: robot pose through the motion model, P <- F P F^T + Q on the
 * robot rows/columns (O(n)). control = {v, omega}. */
int slam_ekfslam_predict(slam_ekfslam* h, const double* control);
/* Batched update with k observed landmarks: ids[k], obs[k x 3] (range,
 * bearing, orientation).  K = P H^T S^-1, mu += K e, P <- P - K (P H^T)^T
 * (a rank-3k update of the lower triangle: the HBM-bound kernel). */
int slam_ekfslam_update(slam_ekfslam* h, int32_t k, const int64_t* ids, const double* obs);
int slam_ekfslam_step(slam_ekfslam* h, const double* control, int32_t k, const int64_t* ids,
                      const double* obs);
/* Device time of the last update (ms): out[5] = {H + P H^T gather, S^-1, K and mu,
 * rank-3k covariance update, 0}. */
int slam_ekfslam_timing(slam_ekfslam* h, double* out);

/* ====================================================================
 * Graph-based SLAM -- replaces TrajectoryEstimator's linearise-and-solve
 * (graph_based_slam.py: setPairObs :362-439, updateEstPose :452-514) and
 * the Gauss-Newton loop of Robot.estimateOpticalTrajectory (:685-715).
 * ==================================================================== */
typedef struct slam_graph slam_graph;

/* One pair of half-edges of the same landmark (HalfEdge :259-300), already
 * ordered as setPairObs orders them (:371-384: "bfr" is the earlier time).
 * The estimate of pose_* is linearised; time_* selects the block of H
 * (its rank among the edge set's times, :478-482) and the pose updated. */
typedef struct {
    int64_t time_bfr, pose_bfr, time_aft, pose_aft;
    double obs_bfr[3];    /* Observation (:20-75): distance, direction, orientation */
    double obs_aft[3];
} slam_graph_edge;

enum { SLAM_GRAPH_AUTO = 0,   /* dense up to 2048 unknowns, PCG above */
       SLAM_GRAPH_DENSE = 1,  /* LU: det, cond and the reference's gate (:494-498) */
       SLAM_GRAPH_PCG = 2 };  /* block-Jacobi PCG on the 3x3 block-sparse H (config 5) */

typedef struct {
    double r_dist;        /* ScanSensor range noise gain (setNoiseParam(5,2,2) :604 -> 0.05) */
    double r_dir;         /* bearing sigma (rad) */
    double r_orient;      /* orientation sigma (rad) */
    double anchor;        /* :475  H[0:3,0:3] += anchor * I  (1e4) */
    double det_min;       /* :496  0.1 < det */
    double cond_max;      /* :496  cond < 1e15 */
    double pcg_tol;       /* PCG: relative residual */
    int32_t pcg_max_iter;
    int32_t solver;       /* SLAM_GRAPH_* */
    double cond_tol;      /* PCG path, cond estimate: a side stops when its Ritz value moved
                             less than cond_tol (relative) over 16 iterations (<= 0: 1e-5) */
    int32_t cond_max_iter;  /* estimate iterations cap (<= 0: 3000) */
    int32_t cond_mode;    /* SLAM_GRAPH_COND_* */
} slam_graph_config;

/* The PCG path's gate (:494-496).  SLAM_GRAPH_COND_ESTIMATE: cond = the extreme
 * eigenvalues of H by LOBPCG on a second stream beside the solve, the
 * reference's `cond < cond_max` from a converged estimate, det not formed
 * (NaN).  SLAM_GRAPH_COND_MARGIN (the Python default; formerly named
 * SLAM_GRAPH_COND_CERTIFY): an estimate with margins, NOT a certificate -- the
 * same estimate stops as soon as its Ritz ratio clears cond_max by a factor 100
 * (or converges: a factor 10; a converged estimate inside that band decides
 * by its own value), and the det half is decided from a log-det interval (M
 * the block diagonal of H, P = M^-1/2 H M^-1/2: [log det M + c(a)(tr P^2 - n),
 * log det M]) whose upper end is rigorous and whose lower end holds unless the
 * estimate's lambda_min over-estimates lambda_min(H) by more than 1000x (a =
 * lambda~min / (1000 max tr M_i)); a half neither decides takes the dense
 * path's value when n <= 2048, else the update is not solved and flagged
 * undecided (slam_graph_gate_info).  SLAM_GRAPH_COND_OFF: no gate
 * (cond NaN, the solve's convergence alone). */
enum { SLAM_GRAPH_COND_ESTIMATE = 0, SLAM_GRAPH_COND_OFF = 1, SLAM_GRAPH_COND_MARGIN = 2,
       SLAM_GRAPH_COND_CERTIFY = SLAM_GRAPH_COND_MARGIN /* former name of the same mode */ };

int slam_graph_create(const slam_graph_config* cfg, int device, slam_graph** out);
int slam_graph_destroy(slam_graph* h);
/* TrajectoryEstimator's pose list (mPosesEst): n_poses x 3. */
int slam_graph_set_poses(slam_graph* h, int64_t n_poses, const double* poses);
int slam_graph_get_poses(slam_graph* h, double* poses);
/* The pairs setPairObs received (builds the block structure once). */
int slam_graph_set_edges(slam_graph* h, int64_t n_edges, const slam_graph_edge* edges);
/* updateEstPose: linearise every edge at the current poses, assemble H and
 * b, gate, solve, update the poses.  stats[4] = {is_calc, sum delta^2, det,
 * cond} (:514).  On the PCG path det is NaN (not formed at this size) and cond
 * is the LOBPCG estimate lambda_max / lambda_min of H (inf when H is not
 * positive definite; NaN with SLAM_GRAPH_COND_OFF): is_calc = 1 means PCG
 * converged with positive curvature and a converged estimate gave cond <
 * cond_max (:496), 0 that the gate rejected H -- including an estimate that
 * reached cond_max_iter unconverged (cond_info status 3: its ratio only bounds
 * cond from below) -- or PCG hit pcg_max_iter (poses unchanged either way). */
int slam_graph_update(slam_graph* h, double* stats);
/* estimateOpticalTrajectory's loop: update until sum delta^2 < delta_sum_th
 * (:692-706) or max_iter; stats: max_iter x 4 (or NULL).  Returns
 * SLAM_ERR_SOLVE (with *n_iter set) when a PCG solve fails to converge. */
int slam_graph_optimize(slam_graph* h, double delta_sum_th, int32_t max_iter, double* stats,
                        int32_t* n_iter);
/* The last assembled system: times (n_times), H (3n_times squared, dense, or
 * NULL), b (3 n_times or NULL), blocks (n_edges x 42: BB, BA, AB, AA, b_B, b_A
 * or NULL).  n_times may be queried with everything else NULL. */
int slam_graph_get_system(slam_graph* h, int64_t* n_times, int64_t* times, double* H, double* b,
                          double* blocks);
/* The block-sparse H of the last update (block rows/columns are time ranks,
 * vals: n_slots x 9 row-major 3x3) and its solution delta (3 n_times);
 * n_slots may be queried with the arrays NULL. */
int slam_graph_get_bsr(slam_graph* h, int64_t* n_slots, int64_t* rows, int64_t* cols, double* vals);
int slam_graph_get_delta(slam_graph* h, double* delta);
/* Device time of the last update (ms): out[5] = {linearise, assemble, solve,
 * pose update, PCG iterations}. */
int slam_graph_timing(slam_graph* h, double* out);
/* The last PCG-path update's cond estimate: out[7] = {iterations, status (1
 * converged, 2 stopped early: cond >= cond_max for certain, 3 cond_max_iter
 * reached, 4 not positive definite), lambda_min, lambda_max, iterations of the
 * min side, of the max side, device time (ms)}.  Zeros after a dense update. */
int slam_graph_cond_info(slam_graph* h, double* out);
/* The last PCG-path update's gate (SLAM_GRAPH_COND_MARGIN): out[14] =
 * {decided by (1 the estimate with its margins and the log-det bounds, 2 a
 * half by the dense path), det decision (1 passed by the interval's lower end
 * at the 1000x margin / 0 rejected by its (rigorous) upper end, 3 / 2 by the
 * dense LU det, -1 undecided: not solved), cond decision (1 passed / 0
 * rejected by the estimate with its margin, 5 passed by a converged estimate
 * inside the margin band, 3 / 2 by the dense Lanczos cond, -1 undecided), log
 * det H lower end, upper end, cond (the value the decision used),
 * lambda_min(H), lambda_max(H) (the estimate's Ritz values), tr(P^2), n,
 * estimate iterations, host ms, det margin (the largest factor by which the
 * Ritz lambda_min may over-estimate lambda_min(H) with the lower end still
 * above ln det_min; 0 if none), cond margin (cond_max / cond)}.  Zeros after a
 * dense update, in the other modes, and when the estimate rejected H for
 * certain (cond_info status 2 / 4). */
int slam_graph_gate_info(slam_graph* h, double* out);
/* HalfEdge (graph_based_slam.py:259-300) with its Observation (:20-75). */
typedef struct {
    int64_t time, pose, landmark;
    double obs[3];        /* distance, direction, orientation */
} slam_graph_half;

/* Robot.estimateOpticalTrajectory's pairing (:697-703): for every landmark id
 * in 0..n_landmarks-1, each 2-combination of its half-edges in recording
 * order (itertools.combinations), ordered as setPairObs orders it (:371-384:
 * the later time is "aft", ties keep the combination order).  Half-edges of
 * other landmark ids never pair.  The half-edges are grouped per landmark on
 * the host (stable, O(n_halves)); the combinations are expanded on the device,
 * one lane per edge.  With edges == NULL only *n_edges is returned; otherwise
 * edges (host, *n_edges records) receives the edge list. */
int slam_graph_pair_halves(int64_t n_halves, const slam_graph_half* halves, int64_t n_landmarks,
                           int device, int64_t* n_edges, slam_graph_edge* edges);
/* One-shot form: poses in/out, stats[4] as slam_graph_update. */
int slam_graph_linearize_solve(const slam_graph_config* cfg, const slam_graph_edge* edges,
                               int64_t n_edges, double* poses, int64_t n_poses, double* stats,
                               int device);

/* ====================================================================
 * ScanSensor.scan (graph_based_slam.py:128-172) over poses x landmarks.
 * yaw_cs[p] = (cos(yaw), sin(yaw), yaw) with yaw = BASE_ANG - theta_p (NumPy's
 * values); tan_scan = tan(BASE_ANG - scan angle).  detect / obs are p-major
 * [n_poses][n_landmarks] (flag; dist, dir, orient).  slam_scan_noise adds the
 * reference's noise to n observations from 3n standard normals in its draw
 * order (dist, dir, orient per detected landmark).
 * ==================================================================== */
int slam_scan_detect(int64_t n_poses, const double* poses, const double* yaw_cs, int64_t n_landmarks,
                     const double* landmarks, double range, double tan_scan, int32_t* detect,
                     double* obs, int device);
int slam_scan_noise(int64_t n, const double* clean, const double* normals, double r_dist,
                    double r_dir, double r_orient, double* out, int device);

/* ErrorEllipse.calc_error_ellipse (mylib/error_ellipse.py:39-55) over n 2x2
 * covariances (row-major [n][4]): out[n][3] = (major, minor, angle); chi from
 * the chi-squared table on the host; column_vectors = 0 keeps the reference's
 * vec[idxmax] row quirk (:51). */
int slam_error_ellipse(int64_t n, const double* covs, double chi, int32_t column_vectors,
                       double* out, int device);

/* ====================================================================
 * NumPy's legacy RandomState stream on the device (MT19937 + polar
 * Box-Muller with the cached normal): the reference's noise source
 * (particle_filter.py:152, :165, :214; motion_model.py:46-48), drawn
 * bit-identically.  State = np.random.get_state()[1:5]: key[624], pos,
 * has_gauss, cached_gaussian.  log() is glibc's, restated with the table of
 * this process's libm (checked against its log() on first use).
 * ==================================================================== */
typedef struct slam_mt slam_mt;
int slam_mt_create(const uint32_t* key, int32_t pos, int32_t has_gauss, double gauss, int device,
                   slam_mt** out);
int slam_mt_destroy(slam_mt* h);
int slam_mt_set_state(slam_mt* h, const uint32_t* key, int32_t pos, int32_t has_gauss, double gauss);
int slam_mt_get_state(slam_mt* h, uint32_t* key, int32_t* pos, int32_t* has_gauss, double* gauss);
/* RandomState.random_sample(n) / standard_normal(n) into host arrays */
int slam_mt_random_sample(slam_mt* h, int64_t n, double* out);
int slam_mt_standard_normal(slam_mt* h, int64_t n, double* out);
/* jump-ahead (host): the 624-word window n_words further along the stream
 * than `window` (word 0's low 31 bits are not part of the MT19937 state and
 * come back unspecified) -- x^n mod the MT19937 characteristic polynomial */
int slam_mt_jump_window(const uint32_t* window, uint64_t n_words, uint32_t* out);
/* glibc's log restated (host; the function the device kernels evaluate) */
int slam_glibc_log(int64_t n, const double* x, double* out);

/* Particle filter with the reference's own noise stream on the device
 * (main_pf, particle_filter.py:86-119): each step draws [rand() if resampling]
 * -> mvn(0, Q, NP) -> mvn(0, R, NL) from the device stream, observes the
 * landmarks from the true pose on the device (__observation :144-154) and runs
 * the estimator.  r_factor = sqrt(s)[:, None] * v of svd(R) (row-major 2x2).
 * truth[4] per step = (x, y, cos(yaw'), sin(yaw')) of the true pose with
 * yaw' = pi/2 - theta (mylib/transform.py:31-35, NumPy's cos / sin). */
int slam_pf_set_rng_mt19937(slam_pf* h, const uint32_t* key, int32_t pos, int32_t has_gauss,
                            double gauss, const double* r_factor);
int slam_pf_get_rng_mt19937(slam_pf* h, uint32_t* key, int32_t* pos, int32_t* has_gauss,
                            double* gauss);
/* the device stream's word ring: out[4] = ring bytes, segments per refill
 * round, words per segment, requests one round feeds (at least) */
int slam_pf_rng_mt19937_info(slam_pf* h, int64_t* out);
int slam_pf_step_truth(slam_pf* h, const double* control, const double* truth, double* z_out,
                       slam_pf_result* res);
/* device-resident batch: truth[n_steps][4]; slam_pf_run then simulates the
 * observations of steps [first, first + k) on the device */
int slam_pf_load_truth(slam_pf* h, int32_t n_steps, const double* truth);

#ifdef __cplusplus
}
#endif
#endif /* SLAM_HIP_H */
