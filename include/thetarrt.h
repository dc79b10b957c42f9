/* thetarrt.h — C-ABI of the MI355X batched RRT-expansion + Theta* line-of-sight engine.
 *
 * The reference (eshira/theta-rrt) has no FFI: its boundary is the Python module surface of
 * rrt.py / search.py with parameters on `builtins`.  Each entry point below replaces
 * one reference call site on the north-star path; the Python mirror in theta-rrt_amd/ binds them via
 * ctypes (theta-rrt_amd/_native.py) and keeps the reference's names and semantics.
 *
 * Conventions
 *   - every function returns int status: 0 = OK, < 0 = error (TR_E_*); tr_last_error() gives a
 *     thread-local message.  No C++ exception crosses the ABI.
 *   - the caller owns every host array; the context owns device memory and pinned staging.
 *   - host-pointer calls are synchronous (outputs valid on return).  `_dev` calls take device
 *     pointers and are asynchronous on the context's stream (tr_set_stream / tr_sync).
 *   - one context per (host thread, GPU); a context is not thread-safe.
 *   - grids are row-major [y][x] bytes, non-zero = free (the reference's `imarray[y][x]`).
 */
#ifndef THETARRT_H
#define THETARRT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TR_OK 0
#define TR_E_ARG (-1)        /* bad argument / shape                                        */
#define TR_E_HIP (-2)        /* HIP runtime failure (message in tr_last_error)              */
#define TR_E_STRAIGHT (-3)   /* drive() on a straight control: the reference's TypeError     */
                             /* (rrt.py:169-171 -> :275 -> :71)                              */
#define TR_E_INDEX (-4)      /* imarray[y][x] outside the array: the reference's IndexError  */
                             /* (non-square maps, search.py:17-33)                          */
#define TR_E_STATE (-5)      /* call order (no grid / no tree / no session)                  */
#define TR_E_VALUE (-6)      /* lazy Theta* re-parent with no closed neighbour: the          */
                             /* reference's ValueError (np.argmin of [], search.py:262)      */

/* Record statuses written by tr_expand_dev (one per sample). */
#define TR_ST_SKIP 0         /* sample not in free space (rrt.py:148-150)                   */
#define TR_ST_COLLISION 2    /* arc/line to qnew hits an obstacle (rrt.py:173-176)           */
#define TR_ST_OK 3           /* expansion accepted                                          */
#define TR_ST_STRAIGHT 4     /* would raise TypeError in the reference                       */
#define TR_ST_INDEX 5        /* would raise IndexError in the reference                      */
#define TR_ST_CONSTRAINT 7   /* steering outside [LEFT, RIGHT] (rrt.py:166-167; dead code)   */
#define TR_FL_DROVE 1        /* qnew came from drive(qnear, u/3) (rrt.py:169-171)            */
#define TR_FL_GOAL 2         /* qnew within tol_xy / tol_ang of the goal (rrt.py:190-201)     */
#define TR_FL_STRAIGHT 4     /* u is the straight control (0, None, None, d)                 */
#define TR_FL_INDEX_SAMPLE 8 /* TR_ST_INDEX raised by the sample's own freespace test         */
#define TR_FL_MEMBER 16      /* the sample is a node of the snapshot: skipped (rrt.py:151)       */
#define TR_FL_SAME_NEAR 32   /* qnew == qnear: the edge is added, cameFrom is not (rrt.py:187)  */

/* builtins parameter block, main.py:14-32 (same names). */
typedef struct tr_params {
  double bikelength, leftconstraint, rightconstraint, frontclearance, maxdrivedist, weightxy,
      xystdv, anglestdv, tol_xy, tol_ang;
  int32_t forwardonly;
  /* 0: a straight control that needs shortening fails the batch with TR_E_STRAIGHT, exactly where
   * the reference raises TypeError (rrt.py:169-171 -> :275).  1: that candidate is discarded like
   * a collision instead (engine extension, off by default; used by long benchmark runs).        */
  int32_t straight_reject;
} tr_params;

/* rand_conf output (rrt.py:68): ((int x, int y), theta). */
typedef struct tr_sample {
  int32_t x, y;
  double th;
} tr_sample;

/* One expansion: qnew pose, control u = (steer, ICC, rad, dist), qnear index. 80 bytes.
 * The expansion also looks the batch up in the snapshot's pose table (rrt.py:151,179,187):
 * TR_FL_MEMBER, TR_FL_SAME_NEAR, and ex = the snapshot node equal to qnew (-1 = a new pose).     */
typedef struct tr_record {
  double x, y, th;
  double steer, iccx, iccy, rad, dist;
  int64_t near;
  int16_t status, flags; /* flags: TR_FL_* */
  int32_t ex;
} tr_record;

/* A record after the device bookkeeping (tr_rrt_pipe_dedupe), as the host replays it: 96 bytes. */
typedef struct tr_resolved {
  tr_record r;
  int64_t idx;           /* final node index of qnew, or -1 when nothing is appended            */
  int32_t flags, pad;    /* TR_RS_*                                                          */
} tr_resolved;
#define TR_RS_MEMBER 1     /* the sample equals a node of the snapshot: skipped (rrt.py:151)     */
#define TR_RS_SAME_NEAR 2  /* qnew == qnear: the edge is added, cameFrom is not (rrt.py:187)      */
#define TR_RS_FIRST 4      /* first occurrence of a new pose: appended as vertex idx (rrt.py:180) */

typedef struct tr_ctx tr_ctx;
typedef struct tr_book tr_book;

const char* tr_last_error(void);
int tr_version(void);

/* ---- context ----------------------------------------------------------------------------- */
int tr_create(int device, tr_ctx** out);
int tr_destroy(tr_ctx* ctx);
/* NULL = the context's own (non-blocking) stream.  Work the caller issues on another stream (e.g.
 * the legacy null stream) is not ordered against the context's: share one explicit stream.
 * Changing the stream waits for the work already issued on the old one.                          */
int tr_set_stream(tr_ctx* ctx, void* hip_stream);
int tr_sync(tr_ctx* ctx);
int tr_set_params(tr_ctx* ctx, const tr_params* p);
/* Engine options, per context (none read from the environment), set while no batch is in flight:
 *   "gate"         1 = the streams of tr_rrt_run hand over through device flags polled by one-wave
 *                  gate kernels, 0 = through HIP events.  tr_create decides it: a two-kernel probe
 *                  checks that kernels of two streams run at the same time, and a context created
 *                  under a tool that serializes every dispatch (rocprofv3 --pmc) starts at 0.
 *   "dd_fused"     1 = the device bookkeeping of a batch is one kernel (default), 0 = three
 *   "dd_fused_max" records per batch up to which the one-kernel form is used (default 8192)
 *   "dd_gatefold"  1 = the next batch's gate rides at the end of the bookkeeping kernel (default)
 *   "fused_delta"  1 = the look-ahead correction runs inside the expansion kernel (default)
 *   "delta_bins"   1 = the bookkeeping kernel files the nodes it appends by map bin and the fused
 *                  correction tests only the bins around each sample (default); 0 = it scans
 *                  every appended node
 *   "nn_grid"      1 = nearest nodes come from cell lists over the map, kept up to date with the
 *                  tree (default; needs a grid); 0 = from a sweep of every node
 *   "nn_far_sweep" global batch size from which the samples far from every node are collected
 *                  and swept as a list instead of scanned by their thread block (default 8193)
 *   "nn_far_nodes" ... those whose second pass covers more nodes than this (default 12288)
 *   "nn_grid_min"  tree size from which they are used (default -1: one node per 8 map pixels)
 *   "book"         1 = the host book follows the device tree (default); 0 = this context only
 *                  keeps the device tree (the ranks of a sharded run that do not report it):
 *                  tr_rrt_book / tr_rrt_findnearest are then not available, goal and raise
 *                  batches still stop the loop on every rank
 *   "trace"        1 = tr_rrt_run prints host timestamps of its last batches to stderr
 * Every setting builds the same tree (tests/test_gpu_bench_parity.py).
 * tr_get_option alone: "head_waits" = batches whose commit slot showed the slot's earlier head
 * when their ready flag arrived (the replay worker then waited for the right one; 0 in every
 * measured run).                                                                                 */
int tr_set_option(tr_ctx* ctx, const char* name, int64_t value);
int tr_get_option(const tr_ctx* ctx, const char* name, int64_t* value);
/* builtins.imarray (main.py:37-42): H = shape[0], W = shape[1]. */
int tr_set_grid(tr_ctx* ctx, const uint8_t* free_yx, int64_t H, int64_t W);

/* ---- device tree mirror (node poses, insertion order = rrt.py G.keys() order) -------------- */
int tr_tree_reset(tr_ctx* ctx, int64_t capacity);
int tr_tree_append(tr_ctx* ctx, const double* xyt, int64_t n); /* host (x, y, theta) triples  */
int64_t tr_tree_size(const tr_ctx* ctx);

/* ---- per-function batches (host arrays, synchronous) --------------------------------------- */
/* NN, rrt.py:155-158: out_idx[j] = first argmin_i L2norm(tree_i, q_j). q_xy int32 pairs.
 * out_d2 (optional, NULL: not wanted): the winner's squared distance, the fp64 sum
 * (qx - x)^2 + (qy - y)^2 that search.py:13-15 takes the square root of.                        */
int tr_nn_batch(tr_ctx* ctx, const int32_t* q_xy, int64_t B, int64_t* out_idx, double* out_d2);
/* lineofsight, search.py:35-41: endpoints (x0, y0, x1, y1) truncated toward zero inside.       */
int tr_los_batch(tr_ctx* ctx, const double* seg4, int64_t n, uint8_t* out);
/* same on device-resident int32 segments (Theta* LOS batches, BASELINE.json cfg4); async.         */
int tr_los_batch_dev(tr_ctx* ctx, const int32_t* d_seg4, int64_t n, uint8_t* d_out);
/* steer, rrt.py:306-541: in (ox, oy, theta, gx, gy, thetagoal) -> out (x, y, theta, steer,
 * iccx, iccy, rad, dist, straight).                                                             */
int tr_steer_batch(tr_ctx* ctx, const double* in6, int64_t n, double* out9);
/* drive, rrt.py:272-304: in (ox, oy, theta, steer, iccx, iccy, rad, dist, straight) -> (x, y,
 * theta); ok[i] = 0 where the reference raises TypeError (straight control).                    */
int tr_drive_batch(tr_ctx* ctx, const double* in9, int64_t n, double* out3, int32_t* ok);
/* bike_clear (mult = 1) / front_of_bike_clear (mult = frontclearance), rrt.py:208-222.         */
int tr_body_clear_batch(tr_ctx* ctx, const double* xyt, int64_t n, double mult, uint8_t* out);
/* all(freespace(px) for px in getArc(begin, land, u)), rrt.py:173-174.  in10 = (bx, by, lx, ly,
 * steer, iccx, iccy, rad, dist, straight).                                                      */
int tr_arc_batch(tr_ctx* ctx, const double* in10, int64_t n, uint8_t* out_clear);

/* findnearest, rrt.py:117-128 (called at main.py:79): for each goal g = (x, y, theta), the child
 * of the first edge, in the reference's traversal `for parent in G.keys(): for child in
 * G[parent]`, with the smallest weightxy * L2norm(child, g) + (1 - weightxy) * |anglediff|.  Edges
 * are (e_par[k], e_child[k]) node indices listing each parent's children in append order (the
 * traversal itself, or the append log); xyt = node poses [n][3].  out_child[g] = node index (-1 when
 * E = 0: the reference's (None, None)), out_dist[g] its distance.  weightxy from tr_set_params.   */
int tr_findnearest_batch(tr_ctx* ctx, const double* xyt, int64_t n, const int64_t* e_par,
                         const int64_t* e_child, int64_t E, const double* goals3, int64_t G,
                         int64_t* out_child, double* out_dist);

/* lineofsight, search.py:35-41, one segment on the host (the grid's host copy, the kernels'
 * closed-form Bresenham): the scalar API call, which a GPU round trip would only slow down.     */
int tr_lineofsight(tr_ctx* ctx, const double* seg4, uint8_t* out);
/* astar, search.py:221-307 (main.py:50): 8-connected A* (thetastar = 0) or lazy Theta* (1) from
 * (sx, sy) to (gx, gy) on the grid, in the reference's order (its priority queue of (f, node)
 * tuples), on the host: one search is a serial chain of pops, each a fraction of a microsecond
 * there.  path_xy receives (x, y) pairs start .. goal, *path_len their count (TR_E_ARG with
 * *path_len = the length needed when cap is short).  stats4 = [expanded (len(closedSet)), 0,
 * line-of-sight tests, status]: status 0 = path found, 1 = start or goal not valid, 2 = start or
 * goal inside an obstacle, 3 = no path (the reference prints / returns False for 1-3).
 * TR_E_VALUE / TR_E_INDEX where the reference raises.                                            */
int tr_astar(tr_ctx* ctx, int64_t sx, int64_t sy, int64_t gx, int64_t gy, int thetastar,
             int64_t* path_xy, int64_t cap, int64_t* path_len, int64_t* stats4);
/* The same search resident on the GPU for a batch of n queries (sx, sy, gx, gy), one wave per
 * query: the open queue (buckets of f in device memory, exact (f, x, y) pop order), gScore,
 * cameFrom, the lazy Theta* line-of-sight test with its re-parent and the path reconstruction all
 * run on the device, and nothing returns to the host before the paths do.  Every query gives what
 * tr_astar gives for it.  path_xy[q * cap * 2 ..] = query q's (x, y) pairs start .. goal,
 * path_len[q] their count (status 7 when cap is short), stats4[q * 4 ..] = [expanded
 * (len(closedSet)), queue entries consumed, pushes that overflowed the queue's buckets, status]: 0 path found, 1 start or goal not valid, 2 inside an
 * obstacle, 3 no path, 4 where the reference raises IndexError, 5 where it raises ValueError
 * (search.py:262), 6 the queue's far list overflowed, 7 path longer than cap.  One query on its own
 * is latency-bound (a few microseconds per pop against the host's fraction of one): tr_astar is the
 * call for a single search, this one for many at once.                                           */
int tr_astar_batch(tr_ctx* ctx, const int32_t* sg4, int64_t n, int thetastar, int64_t* path_xy,
                   int64_t cap, int64_t* path_len, int64_t* stats4);

/* ---- pixel lists in the reference's order (API: search.bresenham / getCircle / getArc) ------ */
int tr_bresenham(tr_ctx* ctx, const double* seg4, int64_t* out_xy, int64_t cap, int64_t* count);
int tr_circle(tr_ctx* ctx, double cx, double cy, double r, int64_t* out_xy, int64_t cap,
              int64_t* count);
int tr_arc_pixels(tr_ctx* ctx, const double* in10, int64_t* out_xy, int64_t cap, int64_t* count);

/* ---- fused batch expansion: the per-iteration body of rrt.py:144-201 for B samples --------- */
/* d_gauss: 3*B legacy gaussians (the np.random stream rand_conf consumes, rrt.py:58,66);
 * goal3 = (gx, gy, gtheta) host.  Every sample reads the device tree as it stands (snapshot).   */
int tr_expand_dev(tr_ctx* ctx, const double* d_gauss, int64_t B, const double* goal3,
                  tr_sample* d_samples, tr_record* d_records);

/* The same expansion for callers that cannot allocate (code under HIP graph capture, tight serving
 * loops, harnesses that forbid hipMalloc).  No counterpart in the reference.  tr_expand_dev keeps
 * its per-batch scratch (query pixels, live flags, nearest nodes, the NN screen's chunk minima) in
 * context buffers that grow on demand; this entry point uses a static 16 MiB device array instead
 * and calls no hipMalloc / hipFree or other allocating routine.  Same arguments, same results.
 * Limit: the scratch of B samples against the tree must fit 16 MiB (e.g. 8192 samples against
 * 262144 nodes); larger calls fail with TR_E_ARG and a message.  Every context on a GPU shares
 * that GPU's array: calls that overlap on one GPU (other contexts, other streams) race; calls on
 * one context's stream are ordered.  Not while a tr_rrt_pipe_stage look-ahead is pending.        */
int tr_expand_dev_noalloc(tr_ctx* ctx, const double* d_gauss, int64_t B, const double* goal3,
                          tr_sample* d_samples, tr_record* d_records);

/* ---- host bookkeeping (no GPU needed): dict G + cameFrom of rrt.py:134-138, 179-188 -------- */
int tr_book_create(tr_book** out);
int tr_book_destroy(tr_book* b);
int tr_book_reset(tr_book* b, const double* start_xyt);
int tr_book_set_straight_reject(tr_book* b, int on);  /* see tr_params.straight_reject */
/* Append records in order (snapshot = first n_snap nodes): membership skip, vertex dedupe, edge,
 * cameFrom, goal stop.  *n_new = nodes appended; *sol = goal node index or -1.                 */
int tr_book_ingest(tr_book* b, const tr_sample* s, const tr_record* r, int64_t n, int64_t n_snap,
                   int64_t* n_new, int64_t* sol);
/* Capacity (pre-faulted host memory) for nodes / edges. */
int tr_book_reserve(tr_book* b, int64_t nodes, int64_t edges);
/* Replay n device-resolved records in order (what tr_rrt_pipe_commit does with a batch). */
int tr_book_replay(tr_book* b, const tr_resolved* rs, int64_t n, int64_t* n_new, int64_t* sol);
int64_t tr_book_size(const tr_book* b);
int64_t tr_book_edges(const tr_book* b);
int tr_book_nodes(const tr_book* b, int64_t from, int64_t to, double* xyt);
/* parent[n] (-1 = None), u6[n*6] (steer, iccx, iccy, rad, dist, straight), CSR children.       */
int tr_book_export(const tr_book* b, int64_t* parent, double* u6, int64_t* e_off, int64_t* e_child);

/* ---- RRT session (rrt.py:130-206) -------------------------------------------------------------
 * The tree lives on the device: a batch's accepted records are deduplicated and numbered there
 * (exact-value pose table, first occurrence in sample order) and new nodes appended on the GPU;
 * the host book replays each batch in sample order (edges, cameFrom, goal) from pinned copies.
 * Batches therefore never wait for the host:
 *   for b: pipe_expand(b) [+ all-gather of the records of every rank] ; pipe_dedupe(b) ;
 *          pipe_commit(b - 1)           (commit lags one batch; results equal tr_rrt_step's)   */
int tr_rrt_begin(tr_ctx* ctx, const double* start3, const double* goal3);
int tr_rrt_reserve(tr_ctx* ctx, int64_t nodes, int64_t batch);   /* capacity hints (no stalls) */
/* Samples + NN + steer/drive + arc for B samples (this rank's slice), async.                     */
int tr_rrt_pipe_expand(tr_ctx* ctx, const double* d_gauss, int64_t B, tr_sample* d_samples,
                       tr_record* d_records);
/* Optional look-ahead: a FUTURE batch is expanded (samples, nearest nodes, steer / rays / drive /
 * arc) against the tree as it stands after the latest pipe_dedupe, on a low-priority side stream,
 * overlapping the current batch.  The next pipe_expand with the same (d_gauss, B, d_samples,
 * d_records) then sweeps only the nodes appended since and re-expands only the samples whose
 * nearest node is one of them; results are unchanged.  The buffers must not be ones a batch in
 * flight still uses (rotate three sets).  At most two staged batches, consumed oldest first.
 * Order per batch: pipe_expand(b), pipe_stage(b + 1), pipe_dedupe(b).  A stage whose snapshot is
 * four or more dedupes old when its pipe_expand comes is dropped (the batch is expanded in full). */
int tr_rrt_pipe_stage(tr_ctx* ctx, const double* d_gauss, int64_t B, tr_sample* d_samples,
                      tr_record* d_records);
/* Device bookkeeping of n records in global sample order (all ranks' slices concatenated) and
 * the D2H of their resolution into the next pinned commit slot (6 slots), async.                 */
int tr_rrt_pipe_dedupe(tr_ctx* ctx, const tr_sample* d_samples, const tr_record* d_records, int64_t n);
/* Host replay of the oldest deduplicated batch.  *n_nodes = tree size after it; *sol = goal node
 * or -1.  TR_E_STRAIGHT / TR_E_INDEX where the reference raises.                                 */
int tr_rrt_pipe_commit(tr_ctx* ctx, int64_t* n_nodes, int64_t* sol);
int tr_rrt_pending(const tr_ctx* ctx);                           /* batches not yet committed */
/* findnearest over the session's tree (device-resident poses, the book's edges); every batch must
 * be committed (TR_E_STATE otherwise).                                                          */
int tr_rrt_findnearest(tr_ctx* ctx, const double* goals3, int64_t G, int64_t* out_node,
                       double* out_dist);
/* ---- multi-GPU: one process per GPU, the sample batch sharded in contiguous slices -----------
 * Rank 0 makes an id, the ranks share it (any side channel), every rank calls tr_comm_init.  The
 * context then all-gathers every batch's samples and records over RCCL (xGMI) in rank order on
 * its stream, and all ranks append the same records: the trees stay identical.                  */
int tr_comm_unique_id(uint8_t* id128);
int tr_comm_init(tr_ctx* ctx, int rank, int world, const uint8_t* id128);
/* The same sharded session with the exchange through the host: every all-gather of tr_rrt_run
 * syncs the context stream, copies this rank's `bytes` to pinned host memory `send`, calls fn,
 * which must fill `recv` with every rank's bytes in rank order (world * bytes), and uploads them.
 * For rehearsals and tests of the sharded loop where RCCL cannot run (several ranks on one GPU;
 * a gloo or socket exchange behind fn).  fn returns 0 on success.                             */
typedef int (*tr_host_gather_fn)(void* user, const void* send, void* recv, int64_t bytes);
int tr_comm_init_host(tr_ctx* ctx, int rank, int world, tr_host_gather_fn fn, void* user);
/* The whole pipelined loop in native code: `rows` batches, global batch BT = B * world (B per rank),
 * batch i reading this rank's slice d_gauss[3 BT i + 3 B rank ...] (d_gauss == NULL: the engine
 * draws them from its gaussian stream, tr_rng_set_state); `stage` = look-ahead depth
 * (0 off, 1 or 2 batches ahead, tr_rrt_pipe_stage); d_samples / d_records hold max(2, stage + 1)
 * sets of B (rotating; both NULL: engine-owned), d_records_all two sets of BT (sharded session;
 * NULL: engine-owned; d_samples_all is not used: the records carry the snapshot lookups); commits
 * lag `lag` batches (1..5).  Stops after the batch that reaches the goal (*sol >= 0).  Same
 * results as the call-per-batch loop.  The streams hand over through device flags polled by
 * one-wave gate kernels, or through events where tr_create found that the device does not run two
 * streams' kernels at the same time (option "gate").  Every device-side wait is bounded: after
 * ~30 s it gives up and the run fails with TR_E_STATE.                                           */
int tr_rrt_run(tr_ctx* ctx, const double* d_gauss, int64_t B, int64_t rows, tr_sample* d_samples,
               tr_record* d_records, tr_sample* d_samples_all, tr_record* d_records_all, int lag,
               int stage, int64_t* n_nodes, int64_t* sol);
/* ---- the np.random gaussian stream on the device (rand_conf's draws, rrt.py:58,66) ----------
 * The engine holds a numpy RandomState MT19937 state (np.random.get_state(): key[624], pos,
 * has_gauss, cached gaussian) and draws RandomState.standard_normal's stream from it on the GPU,
 * bit for bit (legacy polar method; glibc's log restated).  tr_rrt_run with d_gauss == NULL draws
 * each batch's 3 BT gaussians this way (one chunk of batches ahead, on its own stream) and leaves
 * the stream after the last batch it used (the one that reached the goal or raised, else the last
 * row); tr_rng_get_state then returns what np.random.get_state() would after the same draws.     */
int tr_rng_set_state(tr_ctx* ctx, const uint32_t* key624, int32_t pos, int32_t has_gauss,
                     double gauss);
int tr_rng_get_state(tr_ctx* ctx, uint32_t* key624, int32_t* pos, int32_t* has_gauss, double* gauss);
/* n gaussians = RandomState.standard_normal(n) into device memory, async on the context stream. */
int tr_rng_gauss_dev(tr_ctx* ctx, int64_t n, double* d_out);

/* Statistics of the last tr_rrt_run (timing enabled): us11 = last batch's tr_last_timings (5),
 * tr_last_nn_timings (3), and the mean over commits of tr_last_host_timings (3), whose [2] is
 * here the host time spent enqueueing a batch (expand, look-ahead, gather, dedupe calls).       */
int tr_last_run_stats(const tr_ctx* ctx, double* us11, int64_t* commits);
/* Mean GPU durations (HIP events on the stream each kernel runs on) over the sampled batches of
 * the last tr_rrt_run with timing level 1 (every 4th staged batch): us5 = [k_nn_pass1, k_nn_resolve
 * (side stream), k_nn_delta, k_expand_arc, device bookkeeping (main stream)]; samples2 = the
 * number of sampled batches [side, main].                                                       */
int tr_last_run_kernel_us(const tr_ctx* ctx, double* us5, int64_t* samples2);
/* One synchronous batch: expand + dedupe + commit.  gauss on host (gauss_on_device = 0) or device. */
int tr_rrt_step(tr_ctx* ctx, const double* gauss, int64_t B, int gauss_on_device, int64_t* n_nodes,
                int64_t* sol);
tr_book* tr_rrt_book(tr_ctx* ctx);
/* GPU time of the last committed batch (HIP events on the context stream), microseconds:
 * [0] nearest node, [1] steer/drive, [2] arc check, [3] device bookkeeping, [4] sum.
 * level 1 times only [0]; level 2 every phase (each event adds a few us of GPU idle).
 * tr_rrt_run at level 1 brackets every 4th staged batch's kernels (tr_last_run_kernel_us);
 * level 3 is level 1 with every batch bracketed (more samples, more event cost).                 */
int tr_enable_timing(tr_ctx* ctx, int level);
int tr_last_timings(const tr_ctx* ctx, double* us5);
/* NN time of the last committed batch (us): [0] staged sweep on the side stream (overlapped),
 * [1] NN on the batch's own path (delta sweep + resolve, or full sweep + resolve), [2] 0.
 * tr_last_run_stats' us11[5..7] hold the same for a tr_rrt_run, except that [5] and [7] average
 * every staged sweep of the run: [5] = k_nn_pass1 + k_nn_resolve, [7] = k_nn_pass1 alone.         */
int tr_last_nn_timings(const tr_ctx* ctx, double* us3);
/* Host wall time of the last commit, microseconds: [0] wait for the batch, [1] replay, [2] -.    */
int tr_last_host_timings(const tr_ctx* ctx, double* us3);

#ifdef __cplusplus
}
#endif
#endif /* THETARRT_H */
