// LDS-packed scoring family: shared argument blocks of eval_cvrp_words
// (eval.hip), eval_cvrp_words2 and eval_cvrp_rows2 (eval_words.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ctx.hpp"
#include "split.hpp"

namespace vrpms {

// Word-interleaved tours (VRPMS_LAYOUT_WORDS): word w of candidate c holds
// tour positions 4w..4w+3 as bytes, at words[w * C + c].
// The same kernel also reads row-major tours in place: word w of candidate
// c is words[w * wstride + c * cstride] (dwords) -- (C, 1) for the words
// layout, (1, ld / 4) for row-major uint8 rows with ld % 4 == 0.
struct WordsArgs {
  FastSplit f;
  const uint32_t* words;  // uint32 [ceil(n/4)][C], or row-major rows (see strides)
  int64_t C;
  int n;
  uint64_t* keys;
  int32_t* sums;
  int32_t* maxs;
  int32_t* unv;
  int64_t wstride;        // dwords between words w and w + 1 of one candidate
  uint32_t cstride;       // dwords between candidates c and c + 1
};

// Ring depth of eval_cvrp_words2 for tours of n customers: the R in [4, 8]
// that wastes the fewest slots on ceil(n/4) words.
int words2_ring(int n);

// Row-major uint8 tours (the vrpms_eval layout, perm_bytes == 1): candidate
// c at perms[c * ld .. c * ld + n), ld % 4 == 0, perms 16-byte aligned.
// eval_cvrp_rows2 stages 1024 * ILP-row tiles through LDS in chunks of CW
// words, so the API layout needs no transpose.
struct RowsArgs {
  FastSplit f;
  const unsigned char* perms;
  int64_t C;
  int n;
  int ld;
  uint64_t* keys;
  int32_t* sums;
  int32_t* maxs;
  int32_t* unv;
};

// Launch eval_cvrp_words2 with ring depth R (4..8) on stream s.
int launch_words2(const vrpms_ctx* ctx, const WordsArgs& w, int R, hipStream_t s);

// Words per row per LDS stage eval_cvrp_rows2 uses beside the packed
// matrix for tours of n customers (16, 8 or 4), or 0 when no tile fits.
int rows2_chunk_words(const vrpms_ctx* ctx, const FastSplit& f, int n);

// Launch eval_cvrp_rows2 on stream s (caller checked rows2_chunk_words > 0).
int launch_rows2(const vrpms_ctx* ctx, const RowsArgs& r, hipStream_t s);


}  // namespace vrpms
