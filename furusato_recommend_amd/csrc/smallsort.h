// Stable sort of up to 8 192 (int32 key >= 0, int32 value) pairs in two
// launches — smallsort.hip.  Internal interface of the BPR seed grouping
// (bpr.hip) and the table-gradient sort of small steps (tablegrad.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace mirec {

constexpr int64_t kSmallSortMax = 8192;

// Workspace bytes for n pairs (the partial ranks: ceil(n / 256) x n int32).
size_t small_sort_workspace(int64_t n);

// keys_out / vals_out = the pairs in ascending key order, equal keys in
// input order (the stable order: bit for bit a stable radix sort's).
// vals_in == nullptr means the identity (value i for pair i).  Keys must be
// >= 0; 0 <= n <= kSmallSortMax.  No host synchronisation, no memset nodes.
hipError_t small_sort_pairs(void *ws, size_t ws_bytes, const int32_t *keys_in, int32_t *keys_out,
                            const int32_t *vals_in, int32_t *vals_out, int64_t n,
                            hipStream_t st);

}  // namespace mirec
