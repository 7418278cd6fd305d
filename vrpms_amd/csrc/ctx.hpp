// Solver context shared by the translation units of libvrpms.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/vrpms.h"

namespace vrpms {

// Where the kernels read the duration matrix from (SURVEY.md §8d tiers).
enum MatTier : int {
  kTierLdsPacked = 0,  // static CVRP, N <= 128: packed u64 {dur | ret,out,dem} in LDS
  kTierLds = 1,        // whole [H][N][N] (u16 or i32) staged in LDS per workgroup
  kTierGlobal = 2,     // L2 / Infinity-Cache resident gathers (u16 or i32)
};

struct Instance {
  int problem = VRPMS_TSP;
  int H = 1, N = 0, K = 1, objective = VRPMS_OBJ_SUM;
  int max_dur = 0, max_dem = 0, min_dem = 0, max_start = 0, min_start = 0, min_cap = 0, max_cap = 0;
  bool uniform_cap = true;
  bool symmetric = false;      // hour slice 0 is symmetric (O(1) 2-opt delta for static TSP)
  bool sym_all = false;        // every hour slice is symmetric (sa_td_kernel: no reverse rows)
  int cap0 = 0;
  // device copies owned by the context
  int32_t* mat32 = nullptr;    // [H][N][N]
  uint16_t* mat16 = nullptr;   // [H][N][N] when max_dur <= 65535
  uint16_t* mat16h = nullptr;  // [N][N][24] hour-minor copy (H = 24, u16; sa_td_kernel rows)
  uint64_t* pack64 = nullptr;  // [N][N] packed static CVRP layout (tier 0)
  int32_t* dem = nullptr;      // [N]
  int32_t* cap = nullptr;      // [K]
  int32_t* start = nullptr;    // [K]
  int pack_w = 0;              // field width of ret/out in the packed hi word
  // "prefix-ret" layout for a uniform fleet (eval_cvrp_packed MODE 1):
  // lo = dem(b) << S + dur(a,b) + ret(b) - ret(a) (mod 2^32), hi = out(b) + ret(b) | dem(b) << S
  uint64_t* pack64p = nullptr;
  uint64_t* pack64w = nullptr;  // pack64p with hi biased by -lim (eval_cvrp_words)
  int pref_S = 0;
  uint32_t pref_lim = 0, pref_smask = 0;
  int tier = kTierGlobal;
  bool use16 = false;
};

}  // namespace vrpms

struct vrpms_ctx {
  int device = 0;
  bool has_instance = false;
  vrpms::Instance inst;
  int num_cus = 256;
  size_t max_lds = 160 * 1024;
  int opt_split_mode = 0;       // VRPMS_OPT_SPLIT_MODE (0 auto, 2 force branchy, 3 no carry form)
  int opt_staged_m = 0;         // VRPMS_OPT_STAGED_M (0 auto, 1, 2 or 3)
  int opt_route_wg_per_cu = 0;  // sa_route_kernel workgroups per CU (0 auto, 1, 2)
  int opt_words_ilp = 0;        // candidates per lane in eval_cvrp_words2 (0 auto = 2; 1 A/B builds)
  int opt_words_lookahead = 0;  // VRPMS_OPT_WORDS_LOOKAHEAD (words2 gather lookahead, A/B)
  int opt_words_kernel = 0;     // VRPMS_OPT_WORDS_KERNEL (0 auto = words2/rows2, 1 = first generation)
  int opt_ga_fused = 0;          // VRPMS_OPT_GA_FUSED (0 auto, 2 = force the three-kernel GA)
  int opt_sa_route = 0;         // VRPMS_OPT_SA_ROUTE (0 auto, 2 full re-evaluation, 3 route walks, 4 hour rows)
  int opt_rows_config = 0;      // VRPMS_OPT_ROWS_CONFIG (0 auto, 1..5 force eval_cvrp_rows2's (CW, ILP))
  int32_t* d_stats = nullptr;   // scratch for set_instance validation
  uint64_t* d_scratch = nullptr;  // small reduction scratch
  void* search_scratch = nullptr;  // GA children / BF block results (grown on demand)
  size_t search_scratch_bytes = 0;
  void* pool_scratch = nullptr;    // elite selection / island messages (pool.hip, grown on demand)
  size_t pool_scratch_bytes = 0;
  void* comm = nullptr;            // ncclComm_t of the island model (vrpms_island_init)
  int comm_rank = 0, comm_world = 1;
  int opt_island_timeout_s = 120;  // VRPMS_OPT_ISLAND_TIMEOUT_S
  int opt_seg_waves = 0;           // VRPMS_OPT_SEG_WAVES (0 auto, 1..4 force)
  int opt_aco_construct = 0;       // VRPMS_OPT_ACO_CONSTRUCT (0 auto, 2 = the L2 path)
};

namespace vrpms {
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);
void island_release(vrpms_ctx* ctx);  // pool.hip: communicator + pool scratch
}  // namespace vrpms

#define VRPMS_HIP(call)                                               \
  do {                                                                \
    hipError_t _e = (call);                                           \
    if (_e != hipSuccess) return ::vrpms::hip_fail(_e, #call);        \
  } while (0)
