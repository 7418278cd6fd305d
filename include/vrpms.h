/* vrpms.h -- C ABI of the MI355X (gfx950) vrpms solver core.
 *
 * The reference (metehkaya/vrpms) has no native code and no FFI: its solver
 * slot is the `# TODO: Run algorithm` block of each HTTP handler and the stub
 * `src/solver.py`.  This header is the boundary the Python front-end
 * (`vrpms_amd/solver.py`, which keeps the `src/solver.py` entry points and the
 * handler result dicts) binds through ctypes.  Each entry point names the
 * reference line whose behaviour it supplies.
 *
 * Conventions
 *   - Every function returns 0 (VRPMS_OK) or a negative VRPMS_E* code; the
 *     message is in vrpms_last_error() (thread-local).  No C++ exception ever
 *     crosses this boundary.
 *   - All `d_*` pointers are DEVICE pointers owned by the caller (PyTorch-ROCm
 *     tensors in the Python front-end); the library never frees them.  The
 *     context owns its own scratch and derived matrix layouts.
 *   - `stream` is a hipStream_t (NULL = default stream).  Every call after
 *     vrpms_set_instance is asynchronous on that stream; nothing synchronises
 *     except vrpms_set_instance (validation readback) and vrpms_ctx_destroy.
 *   - Nodes are compact indices: node 0 is the depot (VRP, A1) or the
 *     startNode (TSP, A4); customers are 1..N-1.  Tours are "giant tours":
 *     a permutation of customers without the depot, stored as uint8 (N<=256)
 *     or uint16 rows of `ld` elements.  A CVRP tour may also hold the token
 *     0 any number of times (A10 route separator: it closes the current
 *     vehicle's route and opens the next); `n` then counts tokens.
 *   - Semantics are SURVEY.md Appendix A (frozen in oracle/spec.py).
 */
#ifndef VRPMS_H
#define VRPMS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VRPMS_OK 0
#define VRPMS_EINVAL (-1)   /* bad argument / shape */
#define VRPMS_EHIP (-2)     /* HIP runtime error */
#define VRPMS_ERANGE (-3)   /* A9 overflow guard: clock could exceed int32 */
#define VRPMS_ESTATE (-4)   /* no instance loaded */
#define VRPMS_ENOMEM (-5)
#define VRPMS_ETIMEOUT (-6) /* a collective did not complete within its deadline */

#define VRPMS_TSP 0
#define VRPMS_CVRP 1

#define VRPMS_OBJ_SUM 0 /* primary durationSum, secondary durationMax */
#define VRPMS_OBJ_MAX 1 /* primary durationMax, secondary durationSum */

typedef struct vrpms_ctx vrpms_ctx;

/* Library version, (major << 16) | minor. */
int vrpms_version(void);

/* Thread-local message for the last failing call on this thread. */
const char* vrpms_last_error(void);

/* Create / destroy a solver context bound to HIP device `device`. */
int vrpms_ctx_create(int device, vrpms_ctx** out);
int vrpms_ctx_destroy(vrpms_ctx* ctx);

/* Load an instance (replaces the DB fetch result consumed at
 * api/vrp/ga/index.py:41-42 / api/tsp/ga/index.py:33-34).
 *   problem  VRPMS_TSP or VRPMS_CVRP
 *   d_dur    int32 [H][N][N] durations in minutes (A2/A3), H = 1 or 24
 *   d_demand int32 [N] (demand[0] ignored); NULL for TSP
 *   d_cap    int32 [K] vehicle capacities (api/parameters.py:11); NULL for TSP
 *   d_start  int32 [K] start minutes (api/parameters.py:12; TSP: K = 1 and
 *            d_start[0] = startTime, api/parameters.py:43)
 * Validates non-negativity and the A9 int32 guard (synchronises once).
 * Chooses the on-chip tier (LDS-resident / L2-resident) and builds the
 * packed device layouts used by the kernels. */
int vrpms_set_instance(vrpms_ctx* ctx, int32_t problem, const int32_t* d_dur, int32_t H,
                       int32_t N, const int32_t* d_demand, const int32_t* d_cap,
                       const int32_t* d_start, int32_t K, int32_t objective, void* stream);

/* Batched full evaluation of C candidate giant tours (the scoring half of
 * the hot path; the reference's would-be cost function behind
 * api/{tsp,vrp}/<algo>/index.py's TODO slot).
 *   d_perms   [C][ld] uint8 (perm_bytes=1) or uint16 (perm_bytes=2), n used
 *   d_keys    [C] A8 objective keys (required)
 *   d_sum     [C] durationSum (TSP: duration)  -- nullable
 *   d_max     [C] durationMax (TSP: duration)  -- nullable
 *   d_unv     [C] unvisited customer count     -- nullable */
int vrpms_eval(vrpms_ctx* ctx, const void* d_perms, int32_t perm_bytes, int64_t C, int32_t n,
               int64_t ld, uint64_t* d_keys, int32_t* d_sum, int32_t* d_max, int32_t* d_unv,
               void* stream);

/* Same scoring on the word-interleaved tour layout (VRPMS_LAYOUT_WORDS):
 *   d_words   uint32 [ceil(n/4)][C]; word w of candidate c packs customers
 *             4w..4w+3 (uint8 each, low byte first).  N <= 256.
 * Lane c's loads of word w form one contiguous 256-B wave access, so tours
 * stream HBM -> registers with no LDS staging.  This is the layout the GA
 * breed and ACO construct kernels emit for CVRP with N <= 256, so their
 * children / ants are scored by this kernel (eval_cvrp_words2).  Outputs
 * as vrpms_eval. */
int vrpms_eval_words(vrpms_ctx* ctx, const uint32_t* d_words, int64_t C, int32_t n,
                     uint64_t* d_keys, int32_t* d_sum, int32_t* d_max, int32_t* d_unv,
                     void* stream);

/* Re-layout uint8 rows [C][ld] into the word-interleaved layout. */
int vrpms_rows_to_words(vrpms_ctx* ctx, const uint8_t* d_rows, int64_t C, int32_t n, int64_t ld,
                        uint32_t* d_words, void* stream);

/* Which scoring kernel vrpms_eval picks for these tour buffers:
 * 0 = eval_cvrp_packed (LDS packed matrix + LDS-staged tiles),
 * 1 = eval_tsp_staged, 2 = eval_staged (LDS-staged tours, L2-resident or
 * LDS matrix, depot legs in LDS tables; eval_generic when its tables do not
 * fit the LDS); -1 = no instance. */
int vrpms_eval_path(vrpms_ctx* ctx, int32_t perm_bytes, int64_t ld, const void* d_perms);

/* Context options (kernel-variant overrides for A/B tests and profiling).
 *   VRPMS_OPT_SPLIT_MODE: 0 = auto (branch-free prefix-ret split whenever its
 *   packed layout fits), 2 = force the branchy split in eval_cvrp_packed,
 *   3 = the words kernel's compare form of the fit test instead of the
 *   add's carry (the two give identical keys; tests check both). */
#define VRPMS_OPT_SPLIT_MODE 1
/*   VRPMS_OPT_STAGED_M: candidates interleaved per lane in eval_staged
 *   (0 = auto: 2 for hour-indexed matrices, 1 for static; 1 or 2 force). */
#define VRPMS_OPT_STAGED_M 2
/*   VRPMS_OPT_WORDS_KERNEL: LDS-packed kernel for path 0 of vrpms_eval
 *   (0 = auto: eval_cvrp_rows2; 1 = eval_cvrp_packed, the LDS-tile kernel
 *   also used for heterogeneous fleets, A/B only). */
#define VRPMS_OPT_WORDS_KERNEL 3
/*   VRPMS_OPT_WORDS_ILP: candidates per lane in eval_cvrp_words2 (0 = auto:
 *   2; 2 force; 1 only in libraries built with -DVRPMS_AB, A/B). */
#define VRPMS_OPT_WORDS_ILP 4
/*   VRPMS_OPT_WORDS_LOOKAHEAD: words ahead whose gathers eval_cvrp_words2
 *   keeps in flight (0 = auto, 1 or 2 force; A/B). */
#define VRPMS_OPT_WORDS_LOOKAHEAD 5
/*   VRPMS_OPT_ROWS_CONFIG: eval_cvrp_rows2's (chunk words, candidates per
 *   lane): 0 = auto (fewest chunks that fit the LDS), 1 = (8, 2),
 *   2 = (16, 1), 3 = (4, 2), 4 = (8, 1), 5 = (4, 1); A/B. */
#define VRPMS_OPT_ROWS_CONFIG 6
/*   VRPMS_OPT_GA_FUSED: 0 = auto (the fused one-workgroup-per-island GA
 *   kernel whenever the island fits the LDS), 2 = force the three-kernel
 *   path (breed / score / select launches per generation); A/B. */
#define VRPMS_OPT_GA_FUSED 7
/*   VRPMS_OPT_SA_ROUTE: 0 = auto (static symmetric matrix, every demand
 *   fitting the smallest vehicle: every move priced from per-position prefix
 *   sums, sa_seg_kernel -- one capacity, or per-vehicle capacities with each
 *   route tracked on its vehicle; hour-indexed matrix (H = 24): full walks
 *   whose durations come from 24-hour edge rows cached per tour position in
 *   LDS, sa_td_kernel, any fleet; otherwise windowed SA on an exchangeable
 *   fleet prices moves by route-local walks, sa_route_kernel), 2 = force full
 *   re-evaluation of every move (sa_kernel), 3 = force the route-local walks,
 *   4 = force the hour-row walks; A/B. */
#define VRPMS_OPT_SA_ROUTE 8
/*   VRPMS_OPT_ROUTE_WG_PER_CU: workgroups of sa_route_kernel per CU (0 =
 *   auto: 1 for multi-wavefront chains, whose LDS request is padded past
 *   half the CU so each wavefront has a SIMD to itself -- the pricing walk
 *   is VALU-issue bound, so a lone wavefront steps up to twice as fast --
 *   and as many as fit for one-wavefront chains; 1 or 2 force). */
#define VRPMS_OPT_ROUTE_WG_PER_CU 9
/*   VRPMS_OPT_ISLAND_TIMEOUT_S: deadline in seconds of vrpms_island_init
 *   (default 120): the RCCL communicator is created non-blocking and aborted
 *   when not every rank has joined by then, so a rank that never arrives
 *   yields VRPMS_ETIMEOUT instead of a hang. */
#define VRPMS_OPT_ISLAND_TIMEOUT_S 10
/*   VRPMS_OPT_SEG_WAVES: wavefronts per chain of the segment-priced SA kernel
 *   (0 = auto: moves / 64 up to 4 while every chain's wavefronts stay
 *   resident; 1..4 force, A/B -- the trajectories do not depend on it). */
#define VRPMS_OPT_SEG_WAVES 11
/*   VRPMS_OPT_ACO_CONSTRUCT: 0 = auto (ant construction reads the colony's
 *   weights (tau >> 8) * eta from LDS, staged once per iteration by a
 *   workgroup of up to 16 ants of one colony, whenever N * N * 8 bytes fit;
 *   else from L2), 2 = force the L2 path; A/B -- the tours are the same. */
#define VRPMS_OPT_ACO_CONSTRUCT 12
int vrpms_set_option(vrpms_ctx* ctx, int32_t option, int32_t value);

/* Decode ONE giant tour into the result dict of api/vrp/ga/index.py:49-53
 * (A6/A7): d_vehicle_of[i] = vehicle serving perm position i, or -1 when
 * unvisited; d_route_dur[k] = duration of vehicle k (0 if unused). */
int vrpms_decode(vrpms_ctx* ctx, const void* d_perm, int32_t perm_bytes, int32_t n,
                 int32_t* d_vehicle_of, int32_t* d_route_dur, void* stream);

/* Argmin over C keys: d_out[0] = min key, d_out[1] = smallest index holding
 * it.  Wave64 shuffle reduction + one 64-bit atomicMin pass. */
int vrpms_argmin(vrpms_ctx* ctx, const uint64_t* d_keys, int64_t C, uint64_t* d_out,
                 void* stream);

/* ------------------------------------------------------------------------
 * Search kernels: the algorithms behind api/{tsp,vrp}/{sa,ga,aco,bf}/index.py
 * (each stops at `# TODO: Run algorithm` in the reference).  Tours here are
 * uint16 rows [..][n] (n = N - 1 customers).  Every random choice is
 * Philox4x32-10 keyed by `seed` with counters (step/generation/iteration,
 * chain/island/ant, lane/stream), so oracle/spec.py replays them exactly.
 * ---------------------------------------------------------------------- */

/* Simulated annealing (api/{tsp,vrp}/sa/index.py; knobs: api/parameters.py:26-27
 * declares none, so the front-end supplies defaults).  One wavefront per
 * chain: every step the 64 lanes score 64 Philox-sampled moves (swap /
 * 2-opt / relocate) of the chain's tour, the best (key, lane) is accepted if
 * it is no worse or if (u >> 8) < floor(2^24 exp(-dp * invT)); invT is
 * multiplied by inv_alpha after every step (geometric cooling). */
typedef struct {
  int32_t chains;   /* one wavefront each */
  int32_t steps;    /* steps in this call */
  float inv_t0;     /* 1 / temperature at the first step of this call */
  float inv_alpha;  /* per-step factor on 1/T (1/alpha for T *= alpha) */
  uint64_t seed;
  uint64_t step0;   /* global index of the first step (Philox counter) */
  int32_t window;   /* A11: 0 = moves over the whole tour; W > 0 = the second
                       position within W of the first (large tours) */
  uint32_t window_types; /* A12: move types the window applies to, bit t for
                            type t (1 swap, 2 2-opt, 4 relocate); 0 = all */
  int32_t moves;    /* moves sampled per step: 0 or 64 = one wavefront per chain;
                       64 W (W = 2..8) = W wavefronts per chain, move index
                       lane + 64 w (route-local kernel: window > 0 on a fleet
                       of one capacity and start time).  vrpms_tsp_batch_sa
                       ignores it. */
} vrpms_sa_params;

/* d_cur [chains][n] in/out (cur_key out); d_best/d_best_key in/out (set
 * d_best_key to UINT64_MAX before the first call).  CVRP tours may carry
 * A10 separator tokens (n <= N - 1 + K): the moves then also shift route
 * boundaries (relocating a separator), exchange customers across routes and
 * reverse route sequences. */
int vrpms_sa_run(vrpms_ctx* ctx, const vrpms_sa_params* p, uint16_t* d_cur, uint64_t* d_cur_key,
                 uint16_t* d_best, uint64_t* d_best_key, int32_t n, void* stream);

/* Genetic algorithm (api/vrp/ga/index.py; randomPermutationCount -> pop,
 * iterationCount -> generations, api/parameters.py:18-23).  Per generation:
 * binary tournaments, OX1 crossover, Philox-gated mutation (one move),
 * batched scoring, (mu + lambda) survivors per island. */
typedef struct {
  int32_t islands;
  int32_t pop;          /* 2..4096 */
  int32_t generations;  /* generations in this call */
  uint32_t pmut;        /* mutate iff a Philox word < pmut (pmut/2^32 = probability) */
  uint64_t seed;
  uint64_t gen0;        /* global index of the first generation */
} vrpms_ga_params;

/* d_pop [islands][pop][n] and d_keys [islands][pop] in/out (keys must
 * score d_pop on entry, e.g. by vrpms_eval).  For uniform-fleet CVRP on the
 * packed-LDS instances (N <= 128) one 1024-lane workgroup per island runs
 * all `generations` in LDS (ga_fused.hip) when the island fits beside the
 * matrix (CVRP-100: pop <= 256); otherwise each generation is breed ->
 * score -> select launches, the children emitted in the word-interleaved
 * layout and scored by eval_cvrp_words2 when that kernel applies. */
int vrpms_ga_generation(vrpms_ctx* ctx, const vrpms_ga_params* p, uint16_t* d_pop,
                        uint64_t* d_keys, int32_t n, void* stream);

/* Ant colony (api/{tsp,vrp}/aco/index.py), integer pheromone so every
 * update is exact and order-independent: w_ij = (tau_ij >> 8) * eta_ij,
 * eta_ij = floor(2^24 / (1 + D_ij)^2); tau <- clamp(tau - tau >> evap_shift);
 * the iteration-best ant deposits floor(2^30 / (1 + primary)) per edge --
 * or, every bsf_period-th iteration ((iter + 1) % bsf_period == 0, best-so-far
 * buffers given), the colony's best-so-far does (max-min global-best update:
 * an island migrant injected into the best-so-far then shapes tau). */
typedef struct {
  int32_t colonies;
  int32_t ants;        /* per colony, one wavefront each */
  int32_t evap_shift;  /* rho = 2^-evap_shift */
  uint32_t tau_min, tau_max;  /* tau_max <= 2^31 */
  uint64_t seed;
  uint64_t iter;       /* global iteration index (Philox counter) */
  uint32_t bsf_period; /* 0: the iteration best always deposits */
} vrpms_aco_params;

/* d_tau [colonies][N][N] <- tau0, d_eta [N][N] <- floor(2^24 / (1 + D)^2). */
int vrpms_aco_init(vrpms_ctx* ctx, int32_t colonies, uint32_t tau0, uint32_t* d_tau,
                   uint32_t* d_eta, void* stream);

/* One iteration: construct d_tours [colonies][ants][n] (n = N - 1), score
 * them into d_keys, d_iter_best [colonies][2] = (key, ant), update tau.
 * d_best_tours [colonies][n] / d_best_keys [colonies] (nullable, both or
 * neither): each colony's best-so-far, replaced by its iteration best when
 * strictly better (set the keys to UINT64_MAX before the first call).
 * For CVRP with N <= 256 the ants also emit the word-interleaved layout and
 * are scored by the headline kernel (eval_cvrp_words2). */
int vrpms_aco_iteration(vrpms_ctx* ctx, const vrpms_aco_params* p, uint32_t* d_tau,
                        const uint32_t* d_eta, uint16_t* d_tours, uint64_t* d_keys,
                        uint64_t* d_iter_best, uint16_t* d_best_tours, uint64_t* d_best_keys,
                        int32_t n, void* stream);

/* Brute force (api/{tsp,vrp}/bf/index.py): lexicographic ranks
 * [rank_begin, rank_end) of the permutations of customers 1..n (n <= 15);
 * d_out[0] = min key, d_out[1] = smallest rank holding it (UINT64_MAX if
 * the range is empty).  Multi-GPU: disjoint rank ranges + a min. */
int vrpms_bf_run(vrpms_ctx* ctx, int32_t n, uint64_t rank_begin, uint64_t rank_end,
                 uint64_t* d_out, void* stream);

/* Throughput mode (BASELINE.json config 5: many concurrent TSP requests):
 * R independent static TSP requests, each with its own int32 [N][N] matrix
 * (d_mats [R][N][N], node 0 = start node), ONE WORKGROUP PER REQUEST: 4 SA
 * chains per request from Philox Fisher-Yates starts, moves priced by exact
 * O(1) integer deltas (2-opt re-prices the reversed segment when the matrix
 * is asymmetric).  Uses p->steps, inv_t0, inv_alpha, seed (chains/step0
 * ignored).  Out: d_best_tours [R][N-1], d_best_keys [R].  No instance needed. */
int vrpms_tsp_batch_sa(vrpms_ctx* ctx, const int32_t* d_mats, int32_t R, int32_t N,
                       const vrpms_sa_params* p, uint16_t* d_best_tours, uint64_t* d_best_keys,
                       void* stream);

/* ------------------------------------------------------------------------
 * Populations and the island model.  A pool is a set of
 * tours with their A8 keys: SA chains, a GA population ([islands][pop],
 * each island sorted by (key, index)), or the per-colony bests of ACO.
 * Everything here runs on the device, so the search path issues no torch
 * compute (torch only owns the buffers).
 * ---------------------------------------------------------------------- */
typedef struct {
  uint16_t* tours;   /* [count][n] */
  uint64_t* keys;    /* [count] */
  int32_t count;     /* rows */
  int32_t n;         /* customers per tour */
  int32_t groups;    /* VRPMS_INJECT_SORTED: `groups` sorted groups of count / groups rows */
} vrpms_pool;

/* How migrants enter a pool (vrpms_pool_inject / vrpms_island_exchange). */
#define VRPMS_INJECT_WORST 0  /* migrant e replaces the e-th worst row, by (key desc, index asc) */
#define VRPMS_INJECT_SORTED 1 /* migrant e takes slot count/groups - 1 - e/groups of group
                                 e % groups; every group is re-sorted by (key, index) */
#define VRPMS_INJECT_BETTER 2 /* migrant e replaces row e (< count) when its key is smaller */

/* Start tours (the front-end's initial SA chains / GA population, the
 * bench's candidate batch): row r of `count` is the Philox Fisher-Yates
 * permutation of the tokens 1..n+n_sep -- for i = n+n_sep-1 .. 1 swap t[i]
 * and t[w % (i+1)], w word (i & 3) of philox4x32_10((i >> 2, 0xfffffffe, r,
 * stream_id), seed) -- with tokens above n written as 0 (A10 route
 * separators; n_sep = 0 for plain permutations), as uint8 (tour_bytes 1,
 * n + n_sep <= 255) or uint16 rows of `ld` elements. */
int vrpms_random_tours(vrpms_ctx* ctx, int64_t count, int32_t n, int32_t n_sep, int64_t ld,
                       int32_t tour_bytes, uint64_t seed, uint32_t stream_id, void* d_tours,
                       void* stream);

/* Feasible separator tours for the SA start: row r of d_out [count][n+n_sep]
 * is row r of d_in [count][n] (customers only) with a separator (0) where
 * the loaded instance's greedy split would open the next route (at most
 * n_sep, never before the first customer; route i's capacity is
 * capacities[min(i, K-1)]) and the unused separators appended -- same cost
 * as the input while the fleet lasts (oracle/spec.py insert_separators). */
int vrpms_insert_separators(vrpms_ctx* ctx, const uint16_t* d_in, int64_t count, int32_t n,
                            int32_t n_sep, uint16_t* d_out, void* stream);

/* First-fit start tours (oracle/spec.py pack_separators): each customer of
 * row r of d_in [count][n], in order, joins the first of n_sep + 1 routes
 * with room for it (the last route when none has); d_out [count][n + n_sep]
 * lists the routes in order with one separator between consecutive routes.
 * Packs a fleet with little spare capacity into K routes, where
 * vrpms_insert_separators (next fit) runs out of vehicles on a random order. */
int vrpms_pack_separators(vrpms_ctx* ctx, const uint16_t* d_in, int64_t count, int32_t n,
                          int32_t n_sep, uint16_t* d_out, void* stream);

/* The E best rows of a pool by (key, index), ascending: d_tours [E][n],
 * d_keys [E] (0 < E <= min(count, 1024)). */
int vrpms_pool_elites(vrpms_ctx* ctx, const vrpms_pool* pool, int32_t E, uint16_t* d_tours,
                      uint64_t* d_keys, void* stream);

/* Put E migrants (d_tours [E][n], d_keys [E]) into a pool by `mode`. */
int vrpms_pool_inject(vrpms_ctx* ctx, const vrpms_pool* pool, int32_t mode,
                      const uint16_t* d_tours, const uint64_t* d_keys, int32_t E, void* stream);

/* Island message of E elites of n customers: [E keys u64][E x n tours u16],
 * zero padded to a multiple of 16 bytes.  Returns its size in bytes. */
int64_t vrpms_island_msg_bytes(int32_t E, int32_t n);

/* The E elites of `pool` as one message (d_msg, vrpms_island_msg_bytes). */
int vrpms_island_pack(vrpms_ctx* ctx, const vrpms_pool* pool, int32_t E, void* d_msg,
                      void* stream);

/* The E best of `world` gathered messages (d_msgs = world messages back to
 * back, in rank order) by (key, rank, position in the message). */
int vrpms_island_merge(vrpms_ctx* ctx, const void* d_msgs, int32_t world, int32_t E, int32_t n,
                       uint16_t* d_tours, uint64_t* d_keys, void* stream);

/* RCCL communicator of the island model: rank 0 calls vrpms_island_unique_id
 * (128 opaque bytes), shares them with every rank (the front-end uses its
 * torch.distributed group), and every rank calls vrpms_island_init.  One
 * process per GPU; the communicator runs over xGMI on an MI355X node.  The
 * communicator is created non-blocking with a deadline
 * (VRPMS_OPT_ISLAND_TIMEOUT_S): VRPMS_ETIMEOUT, and no communicator, when
 * the ranks did not all join in time. */
int vrpms_island_unique_id(void* out128);
int vrpms_island_init(vrpms_ctx* ctx, const void* unique_id, int32_t rank, int32_t world);
/* world of the context's communicator, 0 when none was initialised */
int vrpms_island_world(vrpms_ctx* ctx);

/* One migration: the E elites of `src` are packed, all-gathered over the
 * context's RCCL communicator (a local copy when none: world 1), merged by
 * (key, rank, position) and injected into `dst` by `mode` -- every rank ends
 * with the same E migrants.  SA: src = bests, dst = current chains, WORST;
 * GA: src = dst = population, SORTED; ACO: src = dst = colony bests, BETTER.
 * (SURVEY.md §8b names this vrpms_island_exchange(ctx, n_elite, stream); the
 * pools are passed per call instead of being registered in the context.) */
int vrpms_island_exchange(vrpms_ctx* ctx, const vrpms_pool* src, const vrpms_pool* dst,
                          int32_t mode, int32_t E, void* stream);

/* Roofline probe (measurement only): `blocks` x 1024 lanes each issue
 * 4 * iters random ds_read_b64 gathers over a `slots`-entry u64 table staged
 * in LDS -- the measured random LDS-gather ceiling R_gather of SURVEY.md §8d. */
int vrpms_probe_lds_gather(vrpms_ctx* ctx, const uint64_t* d_table, int32_t slots, int32_t iters,
                           int32_t blocks, uint64_t* d_sink, void* stream);

/* Roofline probe (measurement only): `blocks` x 256 lanes each issue
 * 8 * iters random 2-byte global loads over a `slots`-entry uint16 table --
 * the measured L2-gather ceiling of the staged kernels (cfg 3 / cfg 4). */
int vrpms_probe_l2_gather(vrpms_ctx* ctx, const uint16_t* d_table, int32_t slots, int32_t iters,
                          int32_t blocks, uint64_t* d_sink, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* VRPMS_H */
