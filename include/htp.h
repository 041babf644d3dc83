/* htp.h -- C ABI of the MI355X-native headland-turn planner (libhtp.so).
 *
 * Drop-in boundary for the OBCA hot path of AgRoboticsResearch/
 * headland_trajectory_planning.  The reference has no FFI of its own (it is
 * pure Python over CasADi/IPOPT); these entry points replace:
 *
 *   htp_obca_solve_batch   OBCAOptimizer(...).solve()   R/obca_py/optimizer.py:77-138 (NLP
 *                          construction) + :475-571 (nlpsol("ipopt") + solution slicing),
 *                          batched over independent problems.
 *   htp_obca_sizes         the decision-variable / constraint counts printed at
 *                          R/obca_py/optimizer.py:490-498.
 *
 * Ownership: every array is caller-owned.  htp_obca_solve_batch takes HOST
 * pointers (the library stages them to HBM); htp_obca_solve_batch_device takes
 * DEVICE pointers already resident in HBM.  The library owns its workspace.
 * Errors: 0 = OK, < 0 = API error (message via htp_last_error); per-problem
 * solver status in htp_obca_result.status (HTP_STATUS_*).  No exceptions cross
 * the ABI.  One htp_ctx per host thread.
 */
#ifndef HTP_H_
#define HTP_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HTP_NPARAM 24
/* per-problem parameter slots (double params[batch][HTP_NPARAM]) */
enum {
  HTP_P_DT = 0, HTP_P_Q00, HTP_P_Q01, HTP_P_Q10, HTP_P_Q11, HTP_P_R00, HTP_P_R01, HTP_P_R10, HTP_P_R11,
  HTP_P_W00, HTP_P_W11, HTP_P_WHEELBASE, HTP_P_MAXSTEER, HTP_P_MAXV, HTP_P_MAXACC, HTP_P_MAXSR,
  HTP_P_DMIN, HTP_P_XLO, HTP_P_XHI, HTP_P_YLO, HTP_P_YHI, HTP_P_HAS_INIT_CONTROL, HTP_P_HAS_INIT_DUAL
};

enum {
  HTP_STATUS_SUCCESS = 0,            /* IPOPT "Solve_Succeeded" */
  HTP_STATUS_ACCEPTABLE = 1,         /* "Solved_To_Acceptable_Level" */
  HTP_STATUS_MAX_ITER = 2,           /* "Maximum_Iterations_Exceeded" */
  HTP_STATUS_RESTORATION_FAILED = 3, /* "Restoration_Failed" */
  HTP_STATUS_STEP_FAILED = 4,        /* "Error_In_Step_Computation" */
  HTP_STATUS_BAD_INPUT = 5,          /* "Invalid_Problem_Definition" */
  HTP_STATUS_CPUTIME = 6,            /* "Maximum_CpuTime_Exceeded" (option max_cpu_time, device clock) */
  HTP_STATUS_INFEASIBLE = 7,         /* "Infeasible_Problem_Detected" (restoration converged, infeasible) */
  HTP_STATUS_TINY_STEP = 8           /* "Search_Direction_Becomes_Too_Small" */
};

typedef struct htp_ctx htp_ctx;

/* One batch of OBCA problems sharing N (horizon), M obstacles, K bodies and
 * the per-polytope edge counts.  Layouts are row-major, problem-major. */
typedef struct {
  int32_t batch, N, M, K, time_opt;   /* time_opt = (W[1][1] != 0), optimizer.py:109 */
  const int32_t* obs_edges;           /* [M] edges of each obstacle polytope (<= 8)  */
  const int32_t* body_edges;          /* [K] edges of each body polytope (<= 8)      */
  const double* traj;                 /* [batch][N][5] init_traj (x, y, v, theta, steer) */
  const double* obs_A;                /* [batch][sum obs_edges][2]  A of A x <= b    */
  const double* obs_b;                /* [batch][sum obs_edges]                      */
  const double* body_G;               /* [batch][sum body_edges][2] G of G x <= g    */
  const double* body_g;               /* [batch][sum body_edges]                     */
  const double* params;               /* [batch][HTP_NPARAM]                         */
  const double* init_control;         /* nullable [batch][N-1][2]                    */
  const double* init_mu;              /* nullable [batch][N][mu_count]               */
  const double* init_lambda;          /* nullable [batch][N][lambda_count]           */
} htp_obca_batch;

typedef struct {
  double* x;            /* [batch][n_var] optimal decision vector, optimizer.py layout */
  double* objective;    /* [batch] f(x*) (unscaled) */
  int32_t* status;      /* [batch] HTP_STATUS_* */
  int32_t* iterations;  /* [batch] IPM iterations */
  int32_t* n_factor;    /* [batch] KKT factorizations (inertia-correction retries included) */
  double* nlp_error;    /* [batch] final scaled NLP error */
  int32_t* n_resto;     /* nullable [batch] feasibility restoration phases entered */
} htp_obca_result;

/* Sizes of one problem (n_var, n_eq, n_ineq as printed by optimizer.py:490-498)
 * and the solver workspace in doubles. */
int htp_obca_sizes(int32_t N, int32_t M, int32_t K, int32_t time_opt, const int32_t* obs_edges,
                   const int32_t* body_edges, int64_t* n_var, int64_t* n_eq, int64_t* n_ineq,
                   int64_t* ws_doubles);

htp_ctx* htp_create(int32_t device);
void htp_destroy(htp_ctx* ctx);
const char* htp_last_error(htp_ctx* ctx);
/* IPOPT option override by name (e.g. "tol", "max_iter", "max_cpu_time" = seconds per problem on the
 * device wall clock, <= 0 off); 0 = OK */
int htp_set_option(htp_ctx* ctx, const char* name, double value);

/* Host buffers in, host buffers out (synchronous). */
int htp_obca_solve_batch(htp_ctx* ctx, const htp_obca_batch* in, htp_obca_result* out);
/* Device-resident buffers in/out; enqueued on `stream` (hipStream_t, may be
 * NULL = default stream).  Not synchronised. */
int htp_obca_solve_batch_device(htp_ctx* ctx, const htp_obca_batch* in, htp_obca_result* out, void* stream);
/* Average duration (ms) of the last solve kernel measured with hipEvents on
 * the launch stream (used by bench.py for the roofline). */
double htp_last_kernel_ms(htp_ctx* ctx);
 /* Diagnostic: per-problem shader-cycle counters of the last solve, [batch][8]:
 * local sweeps, assembly, stage chain, KKT solves, total, errors+grad_lag, line search, update. */
int htp_last_cycles(htp_ctx* ctx, int64_t* out, int32_t batch);

/* Work queue of problem indices feeding ONE persistent solve launch (no
 * reference counterpart: the reference solves one problem per Python call;
 * this is the batch runtime behind bench.py's multi-GPU work stealing,
 * SURVEY.md 8(e)).  The queue lives in pinned, GPU-coherent host memory: the
 * host appends problem indices and closes it; each wavefront of the running
 * launch claims the next ticket with a device atomic, waits until that ticket
 * is published (or the queue is closed: then it retires), and solves problem
 * items[ticket].  Per-ticket results go to out->objective/status/... [ticket];
 * out->x is indexed by problem.  A wave that waits longer than
 * `max_wait_s` for a ticket retires (status of that ticket stays unwritten). */
typedef struct htp_queue htp_queue;
htp_queue* htp_queue_create(htp_ctx* ctx, int64_t capacity);
void htp_queue_destroy(htp_queue* q);
/* Append problem indices (0 <= pid < batch of the launch); -1 when full / closed. */
int htp_queue_publish(htp_queue* q, const int32_t* pids, int64_t n);
int htp_queue_close(htp_queue* q);
int64_t htp_queue_published(const htp_queue* q);
/* Tickets claimed so far by the launch's waves (a monotone lower bound). */
int64_t htp_queue_claimed(const htp_queue* q);
/* Enqueue the persistent launch on `stream` over the device-resident inputs of
 * `in` (in->batch = number of resident problems); `waves` = wavefronts in the
 * launch (<= 0: as many as fit on the device at once). */
int htp_obca_solve_queue_device(htp_ctx* ctx, const htp_obca_batch* in, htp_queue* q, htp_obca_result* out,
                                void* stream, int32_t waves, double max_wait_s);
/* Wavefronts of the OBCA solve kernel resident on the device at once. */
int32_t htp_obca_resident_waves(htp_ctx* ctx, const htp_obca_batch* in);

/* ---------------------------------------------------------------------------
 * Point formulation (R/obca_py/optimizer_points.py OBCAOptimizer: initialize_manual
 * :52-108, generate_object :193-227, generate_variable :229-255, generate_constrain
 * :257-327, solve :157-191): lambda-only duals, one distance row per vehicle hull
 * vertex, hard start/end states, objective sum du^2 + 20 (v dT)^2.  Same solver,
 * batched; x in optimizer_points.py's variable order (X, U, LAMBDA obstacle-major).
 * Parameters: HTP_P_DT, _WHEELBASE, _MAXSTEER, _MAXV (MAX_VELOCITY), _MAXACC,
 * _MAXSR (MAX_STEER_RATE), _DMIN (MIN_DISTANCE_TO_OBS), _XLO.._YHI (min/max x/y);
 * the Q/R/W slots are ignored (the reference never reads r, q). */
typedef struct {
  int32_t batch, N, M, n_vertices;
  const int32_t* obs_edges;   /* [M] halfspaces of each obstacle = len(obstacle) (<= 8) */
  const double* traj;         /* [batch][N][5] init_guess_path */
  const double* obs_A;        /* [batch][sum obs_edges][2] compute_polytope_halfspaces A */
  const double* obs_b;        /* [batch][sum obs_edges]                                 */
  const double* vertices;     /* [batch][n_vertices][2] get_vehicle_vertices (:35-50)   */
  const double* params;       /* [batch][HTP_NPARAM]                                    */
  const double* init_control; /* nullable [batch][N-1][2]                               */
} htp_obca_points_batch;

int htp_obca_points_sizes(int32_t N, int32_t M, int32_t n_vertices, const int32_t* obs_edges, int64_t* n_var,
                          int64_t* n_eq, int64_t* n_ineq, int64_t* ws_doubles);
/* host buffers in/out (synchronous) */
int htp_obca_points_solve_batch(htp_ctx* ctx, const htp_obca_points_batch* in, htp_obca_result* out);
/* device-resident buffers, enqueued on `stream`; timing via htp_last_kernel_ms */
int htp_obca_points_solve_batch_device(htp_ctx* ctx, const htp_obca_points_batch* in, htp_obca_result* out,
                                       void* stream);

/* ---------------------------------------------------------------------------
 * Warm start -> OBCA initial guess (R/obca_py/util.py get_init_ref_path :62-113
 * with cubic_spline.calc_spline_course :92-112): split at gear changes,
 * re-spline every segment over arc length at ds, v = gear * desired_v,
 * steer = atan(L kappa) (sign-flipped in reverse), headings unwrapped,
 * v = 0 at both ends.  One path per wavefront.  Only xs, ys and dirs are read
 * (the reference ignores the yaw and curvature columns). */
enum { HTP_RP_OK = 0, HTP_RP_OVERFLOW = 1 /* n_rows = rows needed so far */, HTP_RP_BAD_SEGMENT = 2,
       HTP_RP_BAD_INPUT = 3 };
typedef struct {
  int32_t batch, cap_points, cap_rows;  /* cap_points >= points of every path                  */
  const int32_t* path_off;              /* [batch+1] CSR offsets into xs / ys / dirs           */
  const double* xs;
  const double* ys;
  const double* dirs;                   /* +1 forward, -1 reverse                              */
  const double* params;                 /* [batch][3]: WHEEL_BASE, desired_v, ds               */
} htp_refpath_batch;
typedef struct {
  int32_t* status;                      /* [batch] HTP_RP_*                                    */
  int32_t* n_rows;                      /* [batch]                                             */
  double* traj;                         /* [batch][cap_rows][5] x, y, v, theta, steer          */
} htp_refpath_result;
int htp_init_ref_path_batch(htp_ctx* ctx, const htp_refpath_batch* in, htp_refpath_result* out);
int htp_init_ref_path_batch_device(htp_ctx* ctx, const htp_refpath_batch* in, htp_refpath_result* out, void* stream);
double htp_init_ref_path_last_ms(htp_ctx* ctx);

/* ---------------------------------------------------------------------------
 * Reeds-Shepp: all admissible paths between pose pairs, sampled
 * (R/path_planner/utils/reeds_shepp.py calc_all_paths :39-65, called by
 * hybrid_a_star_search.py:248 and safety_forward_path_plan.py:368).
 * Query q = (sx, sy, syaw, gx, gy, gyaw, maxc, step_size).  Output is CSR:
 * paths of query q are [path_offsets[q], path_offsets[q+1]); samples of path p
 * are [point_offsets[p], point_offsets[p+1]).  Path order, lengths, ctypes,
 * sample count and values follow the reference (de-duplication, MAX_LENGTH
 * filter and trailing-zero pop included). */
enum { HTP_RS_SEG_L = 0, HTP_RS_SEG_S = 1, HTP_RS_SEG_R = 2, HTP_RS_SEG_NONE = 3 };
enum {
  HTP_RS_OK = 0,
  HTP_RS_ASSERT = 1,      /* reference raises AssertionError (a path with L < 0.01); no paths returned */
  HTP_RS_OVERFLOW = 2,    /* reference raises IndexError in generate_local_course; no paths returned */
  HTP_RS_CAPACITY = 3     /* return code only: output capacity too small, totals reported */
};

typedef struct {
  int64_t cap_paths, cap_points;  /* in: capacity of the arrays below */
  int64_t n_paths, n_points;      /* out: totals needed/written */
  int64_t* path_offsets;          /* [batch+1] */
  int32_t* status;                /* [batch] HTP_RS_* */
  double* lengths;                /* [cap_paths][5] PATH.lengths (unused entries 0) */
  int8_t* ctypes;                 /* [cap_paths][5] HTP_RS_SEG_* */
  double* L;                      /* [cap_paths] PATH.L */
  int64_t* point_offsets;         /* [cap_paths+1] */
  double *x, *y, *yaw, *cs;       /* [cap_points] PATH.x/.y/.yaw/.cs */
  int8_t* directions;             /* [cap_points] PATH.directions */
} htp_rs_paths;

/* Host buffers (synchronous).  Returns HTP_RS_CAPACITY with n_paths/n_points
 * (and status) filled when a capacity is too small; call again with larger
 * arrays (caps 0 = size query). */
int htp_rs_all_paths_batch(htp_ctx* ctx, int32_t batch, const double* queries, htp_rs_paths* out);
/* Device buffers, enqueued on `stream`.  `totals` (device int64[2]) receives
 * (n_paths, n_points); arrays are written only where they fit the capacities
 * (points beyond cap_points and paths beyond cap_paths are skipped). */
int htp_rs_all_paths_batch_device(htp_ctx* ctx, int32_t batch, const double* queries, htp_rs_paths* out,
                                  int64_t* totals, void* stream);
/* Duration (ms) of the last RS batch (hipEvents around its kernels). */
double htp_rs_last_ms(htp_ctx* ctx);


/* ---------------------------------------------------------------------------
 * Hybrid A* warm-start search (motion_type "King": Reeds-Shepp goal shots),
 * one search per problem of the batch:
 *   HybridAStarSearch(start_pose, goal_pose, config_environment, car_model,
 *                     search_heuristic, motion_type="King", yaw_resolution,
 *                     plan_resolution).hybrid_a_star_search(max_nodes)
 *   R/path_planner/hybrid_a_star_search.py:38-74 (ctor), :497-607 (search),
 * called from R/path_planner/headland_path_planning.py:203-219 and
 * R/test/obca.ipynb:261-272.  The environment and the heuristic are lowered to
 * polygons (host side, headland_trajectory_planning_amd/path_planner):
 *   body      car_model.car_poly (car_model.py:102-120), vertices in the car frame
 *   blockers  orchard_geometry_environment.py tree_polys + obstacle_polys
 *             (check_path_feasibility :423-437)
 *   field     field_range_poly (:374-378, boundary_check=True); -1 = none
 *   lanes     reference_line_heuristic.py segment_lanes (CCW, convex) with
 *             their search_lengths (:84-96); their union is guided_lane
 *   guide     guided_path rows (x, y, yaw, s) (:50-82)
 *   motions   motion steers (steer, direction) (:331-354)
 * Polygons are vertex ranges [poly_off[p], poly_off[p+1]) of `vertices`
 * (no repeated closing vertex).  Per-search descriptor desc[b][HTP_HA_NDESC]
 * holds polygon / guide / motion index ranges into these shared pools. */
#define HTP_HA_NPARAM 16
enum {
  HTP_HA_P_SX = 0, HTP_HA_P_SY, HTP_HA_P_SYAW, HTP_HA_P_GX, HTP_HA_P_GY, HTP_HA_P_GYAW,
  HTP_HA_P_RES,      /* plan_resolution */
  HTP_HA_P_YAWRES,   /* yaw_resolution */
  HTP_HA_P_WB,       /* car_model.WHEEL_BASE */
  HTP_HA_P_MAXSTEER, /* car_model.MAX_STEER */
  HTP_HA_P_CURV,     /* car_model.curvature = tan(MAX_STEER) / WHEEL_BASE */
  HTP_HA_P_DEFLEN,   /* search_heuristic.default_search_length */
  HTP_HA_P_MAXNODES  /* max_nodes */
};
#define HTP_HA_NDESC 12
enum {
  HTP_HA_D_BODY = 0,                   /* polygon id of the body */
  HTP_HA_D_BLK0, HTP_HA_D_BLK1,        /* blocker polygon ids [BLK0, BLK1) */
  HTP_HA_D_LANE0, HTP_HA_D_LANE1,      /* lane polygon ids [LANE0, LANE1) */
  HTP_HA_D_FIELD,                      /* field polygon id or -1 */
  HTP_HA_D_GUIDE0, HTP_HA_D_GUIDE1,    /* guide rows [GUIDE0, GUIDE1) */
  HTP_HA_D_MOT0, HTP_HA_D_MOT1,        /* motion rows [MOT0, MOT1) */
  HTP_HA_D_KING                        /* 1 = King (Reeds-Shepp goal shots), 0 = Pawn (Dubins + spline) */
};
enum {
  HTP_HA_FOUND = 0,            /* goal reached (Reeds-Shepp shot or within one cell) */
  HTP_HA_NO_PATH = 1,          /* open set exhausted ("No solution is available") */
  HTP_HA_MAX_NODES = 2,        /* counter > max_nodes ("drop the planner") */
  HTP_HA_START_GOAL_BLOCKED = 3,
  HTP_HA_RS_ERROR = 4,         /* the reference raises inside reeds_shepp.calc_all_paths */
  HTP_HA_CAPACITY = 5,         /* node pool exhausted (cannot happen with the library's sizing) */
  HTP_HA_BAD_INPUT = 6,        /* a per-search shape check failed (see the limits below); the search is not run */
  HTP_HA_BACKTRACK = 7         /* the reference raises KeyError while backtracking */
};
/* Per-search limits (hastar_core.h valid_search; a search outside them ends HTP_HA_BAD_INPUT on the device and in
 * the host build alike): body polygon 3..HTP_HA_MAX_BODY vertices, at most HTP_HA_MAX_LANES lane polygons and
 * HTP_HA_MAX_MOTIONS motion primitives, and for every search length L (HTP_HA_P_DEFLEN and each lane's lane_len)
 * n = rint(L / HTP_HA_P_RES) with 1 <= n, n + 1 <= HTP_HA_MAX_POSES and nmotions * (n + 1) <= HTP_HA_TRAJ_CAP:
 * one expansion's rollouts are held in LDS.  The reference has no such limit; its planners' settings need at most
 * 14 x 16 = 224 (King, search length 1.5 m at 0.1 m).  King's 14 motions allow n + 1 <= 36 poses per primitive,
 * i.e. L <= 35 res (3.5 m at 0.1 m). */
#define HTP_HA_MAX_BODY 8
#define HTP_HA_MAX_LANES 32
#define HTP_HA_MAX_MOTIONS 16
#define HTP_HA_MAX_POSES 64
#define HTP_HA_TRAJ_CAP 512

typedef struct {
  int32_t batch;
  int32_t npoly, nvert, nguide, nmotion;  /* pool sizes */
  const double* params;     /* [batch][HTP_HA_NPARAM] */
  const int32_t* desc;      /* [batch][HTP_HA_NDESC] */
  const int32_t* poly_off;  /* [npoly+1] */
  const double* vertices;   /* [nvert][2] */
  const double* lane_len;   /* [npoly] search length of lane polygons (others unused) */
  const double* guide;      /* [nguide][4] */
  const double* motions;    /* [nmotion][2] */
  int32_t max_nodes_cap;    /* >= every params[b][HTP_HA_P_MAXNODES] (sizes the node pool) */
  int32_t cap_path;         /* samples per search in the path outputs */
  int32_t cap_log;          /* expansions per search in the expansion log (0 = none) */
} htp_hastar_batch;

typedef struct {
  int32_t* status;      /* [batch] HTP_HA_* */
  int32_t* counter;     /* [batch] the reference's returned node counter */
  int32_t* n_path;      /* [batch] samples of the returned path (may exceed cap_path: then truncated) */
  int32_t* n_expanded;  /* [batch] nodes popped */
  int64_t* n_pose;      /* [batch] footprint poses tested */
  double *x, *y, *yaw, *dir, *k;  /* [batch][cap_path]: xs, ys, yaws, dirs, ks of the search result */
  int32_t* expanded;    /* [batch][cap_log][3] grid index of every popped node (nullable) */
} htp_hastar_result;

/* Host buffers in and out (synchronous). */
int htp_hastar_search_batch(htp_ctx* ctx, const htp_hastar_batch* in, htp_hastar_result* out);
/* Device buffers in and out, enqueued on `stream`. */
int htp_hastar_search_batch_device(htp_ctx* ctx, const htp_hastar_batch* in, htp_hastar_result* out, void* stream);
/* Duration (ms) of the last search kernel (hipEvents on its stream). */
double htp_hastar_last_ms(htp_ctx* ctx);


/* ---------------------------------------------------------------------------
 * Y-type parking grid search: search_y_type_parking_path(car_model, config_env,
 * end_pose, backward_steer_dir, forward_steer_dir, max/min steers and lengths,
 * step_size) R/path_planner/headland_path_planning.py:382-451, one search per
 * problem of the batch.  The grid axes (np.arange values, the reference's loop
 * order: backward length, forward length, backward steer, forward steer) live in
 * `axis`; the first collision-free candidate is returned with its manoeuvre
 * (rows x, y, yaw, k, dir in the odom frame, get_y_type_parking_path +
 * get_path_in_odom :487-527).  Footprint = car_poly at every pose against
 * blockers (obstacle + tree polygons) and inside the field polygon
 * (check_path_feasibility :423-458, boundary_check=True). */
#define HTP_YP_NPARAM 16
enum {
  HTP_YP_P_EX = 0, HTP_YP_P_EY, HTP_YP_P_EYAW,  /* end (row-enter) pose */
  HTP_YP_P_BDIR, HTP_YP_P_FDIR,                 /* backward / forward steer directions (+-1) */
  HTP_YP_P_WB, HTP_YP_P_STEP,                   /* car_model.WHEEL_BASE, step_size */
  HTP_YP_P_R00, HTP_YP_P_R01, HTP_YP_P_R10, HTP_YP_P_R11, HTP_YP_P_TX, HTP_YP_P_TY,  /* states2SE3(end pose) */
  HTP_YP_P_YAW_ODOM                             /* SE32states(T)[5] */
};
#define HTP_YP_NDESC 12
enum {
  HTP_YP_D_BODY = 0, HTP_YP_D_BLK0, HTP_YP_D_BLK1, HTP_YP_D_FIELD,
  HTP_YP_D_BL0, HTP_YP_D_NBL, HTP_YP_D_FL0, HTP_YP_D_NFL, HTP_YP_D_SB0, HTP_YP_D_NSB, HTP_YP_D_SF0, HTP_YP_D_NSF
};
enum { HTP_YP_FOUND = 0, HTP_YP_NONE = 1, HTP_YP_END_BLOCKED = 2, HTP_YP_BAD_INPUT = 3 };

typedef struct {
  int32_t batch, npoly, nvert, naxis;
  const double* params;     /* [batch][HTP_YP_NPARAM] */
  const int32_t* desc;      /* [batch][HTP_YP_NDESC] */
  const int32_t* poly_off;  /* [npoly+1] */
  const double* vertices;   /* [nvert][2] */
  const double* axis;       /* [naxis] grid axis values */
  int32_t cap_path;         /* rows per search in `path` */
} htp_ypark_batch;

typedef struct {
  int32_t* status;   /* [batch] HTP_YP_* */
  int32_t* cand;     /* [batch] index of the chosen candidate in loop order (-1: none) */
  int32_t* n_path;   /* [batch] rows of the chosen manoeuvre */
  double* params;    /* [batch][4] backward length, forward length, backward steer, forward steer */
  int64_t* n_pose;   /* [batch] footprint poses tested (nullable) */
  double* path;      /* [batch][cap_path][5] */
} htp_ypark_result;

int htp_ypark_search_batch(htp_ctx* ctx, const htp_ypark_batch* in, htp_ypark_result* out);
int htp_ypark_search_batch_device(htp_ctx* ctx, const htp_ypark_batch* in, htp_ypark_result* out, void* stream);
double htp_ypark_last_ms(htp_ctx* ctx);

/* ---------------------------------------------------------------------------
 * Orchard scene -> OBCA obstacles: the synthetic orchard
 * of R/path_planner/utils/map_utils.py create_tree_rows :45-61 and the OGE_OBCA
 * obstacle producer, one scene per GPU thread (csrc/oge_core.h):
 *   env = orchard_environment_OBCA(tree_rows, [], tree_width, headland_width)
 *   boundary = env.create_boundary_polygons()          OGE_OBCA.py:306-373
 *   rows = env.get_obstacle_tree_rows(start, end)      :477-591
 *   obstacles = env.get_obstacles_for_OBCA(boundary, rows, start, end, side)  :593-677
 * and, per obstacle, compute_polytope_halfspaces as R/obca_py/optimizer.py:184-186
 * calls it (A x <= b, cdd row normalisation, 7-decimal rounding).  The reference's
 * np.random draws are inputs (row_draws: create_tree_rows' uniform(-l_std, l_std)
 * per row; eps_draws: create_headland_countour_lines' uniform(-0.5, 0.5) per row,
 * orchard_geometry_environment.py:71).  Polygons come out in the reference's order. */
#define HTP_OGE_NPARAM 16
enum {
  HTP_OGE_P_NROWS = 0,   /* tree rows (3..32) */
  HTP_OGE_P_ROWW, HTP_OGE_P_ROWLEN, HTP_OGE_P_SLOPE,   /* create_tree_rows row_width, row_lengths, slope_angle */
  HTP_OGE_P_TREEW, HTP_OGE_P_HW,                       /* tree_width, headland_width */
  HTP_OGE_P_SX, HTP_OGE_P_SY, HTP_OGE_P_SYAW,          /* start (row-leave) pose */
  HTP_OGE_P_EX, HTP_OGE_P_EY, HTP_OGE_P_EYAW,          /* end (row-enter) pose */
  HTP_OGE_P_SIDE                                       /* 1 NEAR_SIDE, -1 FAR_SIDE */
};
#define HTP_OGE_MAXROWS 32
#define HTP_OGE_MAXPOLY 32
#define HTP_OGE_MAXV 12
enum { HTP_OGE_OK = 0, HTP_OGE_BAD_INPUT = 1, HTP_OGE_NO_ROW_BETWEEN = 2 /* reference: IndexError */,
       HTP_OGE_OVERFLOW = 3 /* more than MAXPOLY polygons or MAXV vertices */, HTP_OGE_EMPTY_SIDE = 4 };
typedef struct {
  int32_t batch, max_rows;  /* max_rows = row stride of the draw arrays */
  const double* params;     /* [batch][HTP_OGE_NPARAM] */
  const double* row_draws;  /* [batch][max_rows] */
  const double* eps_draws;  /* [batch][max_rows] */
} htp_oge_batch;
typedef struct {
  int32_t* status;          /* [batch] HTP_OGE_* */
  int32_t* n_poly;          /* [batch] */
  int32_t* n_vert;          /* [batch][MAXPOLY] */
  double* vertices;         /* [batch][MAXPOLY][MAXV][2] */
  int32_t* n_facet;         /* [batch][MAXPOLY] facets (-1: fewer than 3 distinct vertices) (nullable) */
  double* A;                /* [batch][MAXPOLY][MAXV][2] (nullable with n_facet) */
  double* b;                /* [batch][MAXPOLY][MAXV]    (nullable with n_facet) */
} htp_oge_result;
int htp_oge_obstacles_batch(htp_ctx* ctx, const htp_oge_batch* in, htp_oge_result* out);
int htp_oge_obstacles_batch_device(htp_ctx* ctx, const htp_oge_batch* in, htp_oge_result* out, void* stream);
double htp_oge_last_ms(htp_ctx* ctx);

/* ---------------------------------------------------------------------------
 * Classic headland turns: one warm-start path per problem,
 * rows [x, y, yaw, k, dir] as the reference's planners return them (csrc/classic_core.h):
 *   HTP_CT_DUBINS      get_dubins_path_full(start, end, R, step)   safety_forward_path_plan.py:286-297
 *   HTP_CT_CIRCLEBACK  get_circle_back_path_full(start, end, R, car, side, step)   :395-454
 *   HTP_CT_FISHTAIL    get_start_end_pose_for_reeds_shepp (:300-364) + the collision-free Reeds-Shepp word
 *                      with the least backward length + Dubins lead-in/out (R/test/classic_planner.ipynb 10-11)
 * Footprints (fish-tail only): the body polygon at every pose against the blocker polygons
 * (check_path_feasibility :423-458, boundary_check=False); polygons in CSR pools as for the searches. */
#define HTP_CT_NPARAM 12
enum { HTP_CT_P_TYPE = 0, HTP_CT_P_SIDE,                      /* HTP_CT_* ; map_utils NEAR_SIDE 1 / FAR_SIDE 2 */
       HTP_CT_P_SX, HTP_CT_P_SY, HTP_CT_P_SYAW, HTP_CT_P_EX, HTP_CT_P_EY, HTP_CT_P_EYAW,
       HTP_CT_P_WB, HTP_CT_P_MAXSTEER, HTP_CT_P_RADIUS, HTP_CT_P_STEP };
enum { HTP_CT_DUBINS = 0, HTP_CT_CIRCLEBACK = 1, HTP_CT_FISHTAIL = 2 };
enum { HTP_CT_OK = 0, HTP_CT_OVERFLOW = 1, HTP_CT_NO_WORD = 2 /* no collision-free word (reference: None) */,
       HTP_CT_BAD_INPUT = 3, HTP_CT_RS_ERROR = 4 /* reference raises in reeds_shepp */, HTP_CT_NO_DUBINS = 5 };
typedef struct {
  int32_t batch, npoly, nvert;
  const double* params;     /* [batch][HTP_CT_NPARAM] */
  const int32_t* desc;      /* [batch][3]: body polygon id, blockers [blk0, blk1) */
  const int32_t* poly_off;  /* [npoly+1] */
  const double* vertices;   /* [nvert][2] */
  int32_t cap_path;         /* rows per problem in `path` */
  int32_t cap_samples;      /* Dubins samples per piece (scratch sizing) */
} htp_classic_batch;
typedef struct {
  int32_t* status;          /* [batch] HTP_CT_* */
  int32_t* n_path;          /* [batch] */
  double* path;             /* [batch][cap_path][5] x, y, yaw, k, dir */
} htp_classic_result;
int htp_classic_turn_batch(htp_ctx* ctx, const htp_classic_batch* in, htp_classic_result* out);
int htp_classic_turn_batch_device(htp_ctx* ctx, const htp_classic_batch* in, htp_classic_result* out, void* stream);
double htp_classic_last_ms(htp_ctx* ctx);

/* ---------------------------------------------------------------------------
 * Orchard workload chain on the device (synth.make_orchard_instance's steps after the scene draws): for each
 * problem, the classic turn (htp_classic_turn_batch) -> get_init_ref_path at spacing ds / 2 = L / (2N - 2)
 * (ds = L / (N - 1), the resampled spacing), desired_v = min(ds / dT, 0.9) (R/obca_py/util.py:62-113) -> the init guess resampled to N rows and the
 * headland width the warm start needs -> the OGE_OBCA obstacle producer (htp_oge_obstacles_batch) -> quads,
 * the M nearest, halfspaces.  Writes the htp_obca_batch arrays traj / obs_A / obs_b (4 edges per obstacle)
 * in HBM, enqueued on `stream`; intermediates live in the context.  `scenes` and `turns` hold device
 * pointers; scenes.params[b][HTP_OGE_P_HW] is overwritten with the chain's headland width. */
typedef struct {
  int32_t batch, N, M;
  htp_oge_batch scenes;            /* device */
  htp_classic_batch turns;         /* device pools */
  const double* margin;            /* [batch] device: boundary margin behind the warm start */
  int32_t n_vpoly;                 /* vehicle footprint polygons (car frame): body, then the implement (<= 2) */
  int32_t vpoly_nv[2];
  double vpoly[2][8][2];
  double dT, wheel_base;
  int32_t cap_rows;                /* init-guess rows per problem */
  double* traj;                    /* [batch][N][5] device out */
  double* obs_A;                   /* [batch][4 M][2] device out */
  double* obs_b;                   /* [batch][4 M] device out */
  int32_t* status;                 /* [batch] device out: 0, or 16 * stage + that stage's status
                                      (stage 1 classic, 2 init guess, 3 obstacle producer, 4 quads) */
} htp_chain_batch;
int htp_orchard_chain_device(htp_ctx* ctx, const htp_chain_batch* in, void* stream);
double htp_chain_last_ms(htp_ctx* ctx);


/* ---------------------------------------------------------------------------
 * The notebook planner chain on the device (R/path_planner/headland_path_planning.py:124-255, the planner of
 * R/test/obca.ipynb cells 9-15): for each problem, the Y-type parking search (htp_ypark_search_batch_device)
 * fixes the intermediate pose; the heuristic lowering (csrc/ychain_core.h: get_topology_waypoints, the
 * ReferenceLineHeuristic guide path, segment lanes and search lengths) writes the hybrid A* inputs of that
 * problem into reserved slots of the search's pools; the hybrid A* search (htp_hastar_search_batch_device) runs
 * from the start to the intermediate pose; its path and the parking manoeuvre are joined and turned into the
 * init guess (get_init_ref_path, refpath_core.h) and resampled to N rows (the OBCA solve's traj input).
 * Everything stays in HBM; four launches on `stream`.  Reserved hybrid A* slots of problem b: polygon ids
 * [lane_poly0 + b * HTP_YC_POLY_STRIDE, + HTP_YC_POLY_STRIDE) (the last one spans the unused vertices),
 * vertices [lane_vert0 + b * HTP_YC_VERT_STRIDE, ...), guide rows [guide0 + b * guide_stride, ...); the host
 * sets hastar.poly_off at every problem's first slot id (and at lane_poly0 + batch * HTP_YC_POLY_STRIDE), the
 * device writes the rest, hastar.params[b] GX..GYAW and hastar.desc[b] LANE0..GUIDE1. */
#define HTP_YC_MAXWP 10
#define HTP_YC_POLY_STRIDE HTP_YC_MAXWP
#define HTP_YC_VERT_STRIDE ((HTP_YC_MAXWP - 1) * 80)
typedef struct {
  int32_t batch, N;
  htp_ypark_batch ypark;            /* device arrays */
  htp_ypark_result ypark_out;       /* device arrays (path: [batch][ypark.cap_path][5]) */
  htp_hastar_batch hastar;          /* device pools; the lane / guide slots and GX..GYAW, LANE0..GUIDE1 are written */
  htp_hastar_result hastar_out;     /* device arrays (paths: [batch][hastar.cap_path]) */
  const double* rows;               /* [batch][max_rows][4]: near x, near y, far x, far y of every tree row */
  const int32_t* nrows;             /* [batch] */
  const double* eps;                /* [batch][max_rows]: check_side_of_a_point's uniform(-0.5, 0.5) draws */
  const double* start;              /* [batch][3] the search start pose */
  int32_t max_rows;
  double drive_row_offset;          /* headland_planner_y_type_park's drive_row_offset */
  int32_t lane_poly0, lane_vert0, guide0, guide_stride;
  const double* rp_params;          /* [batch][3] WHEEL_BASE, desired_v, ds (get_init_ref_path) */
  int32_t cap_rows;                 /* init-guess rows per problem */
  double* ref;                      /* [batch][cap_rows][5] init guess out (get_init_ref_path rows) */
  int32_t* n_ref;                   /* [batch] */
  double* traj;                     /* [batch][N][5] the init guess resampled to N rows (OBCA traj) */
  int32_t* status;                  /* [batch]: 0, or 16 * stage + that stage's status (1 Y-park, 2 lowering,
                                       3 hybrid A*, 4 init guess) */
} htp_ychain_batch;
int htp_ypark_hastar_chain_device(htp_ctx* ctx, const htp_ychain_batch* in, void* stream);
/* Per-stage kernel times (ms) of the last chain: Y-park, lowering, hybrid A*, init guess + resample. */
int htp_ychain_last_ms(htp_ctx* ctx, double* ms4);

/* ---- deterministic double-double libm of the planner cores (csrc/htp_libm.h) ----------------------------------------
 * Replaces nothing in the reference: the reference's planners call CPython's math module / numpy (glibc, or
 * numpy's SIMD kernels), whose last bits differ between platforms.  Every device planner kernel and every host
 * build of the same cores evaluates sin, cos, tan, atan, atan2, asin, acos, hypot and pow with this one
 * double-double implementation (< 2^-100 relative before one final rounding, no Ziv fallback; the same
 * operations on both sides, so the same doubles), so integer outputs that hang on the last bit (a spline piece's sample
 * count, R/path_planner/utils/cubic_spline.py:102) are identical on the GPU and on the host.
 * fn: 0 sin, 1 cos, 2 tan, 3 atan, 4 atan2(x[i], y[i]), 5 asin, 6 acos, 7 hypot(x[i], y[i]), 8 pow(x[i], y[i]), 9 log; the solver's
 * fast deterministic functions (htp_fastm.h, <= 2 ulp): 10 log, 11 sin, 12 cos, 13 tan.
 * x, y, out: device arrays of n doubles (y only for the two-argument functions). */
int htp_libm_batch_device(htp_ctx* ctx, int32_t fn, const double* x, const double* y, double* out, int64_t n,
                          void* stream);

/* The fp64 matrix-core op of the solver's Riccati recursion (v_mfma_f64_16x16x4f64) on n caller tiles:
 * D[t] = A[t] (16x4, row-major) * B[t] (4x16, row-major) + C[t] (16x16, row-major), device arrays.  A
 * diagnostic surface with no reference counterpart: it pins the host model of the op's rounding that the
 * bit-exact host emulation of the device solver uses (tests/test_gpu_mfma_model.py). */
int htp_mfma_f64_probe(htp_ctx* ctx, const double* A, const double* B, const double* C, double* D, int64_t n,
                       void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HTP_H_ */
