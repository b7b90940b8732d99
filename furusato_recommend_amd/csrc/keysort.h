// Stable counting sort of (int32 key, int32 value) pairs whose keys are dense
// ids in [0, nk) — keysort.hip.  Internal interface of the table-gradient key
// sorts (tablegrad.hip); the C ABI (mirec_key_sort_*) wraps the same calls.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace mirec {

// Largest n the sort takes (the bucket-class bounds keep every LDS table
// within 64 KB below it).
constexpr int64_t kKeySortMaxN = (int64_t)1 << 27;

// Workspace bytes for n pairs over nk buckets (0 < nk < 2^31).
size_t key_sort_workspace(int64_t n, int32_t nk);

// keys_out / vals_out = the pairs in ascending key order, equal keys in input
// order (bit for bit what a stable radix sort returns).  vals_in == nullptr
// means the identity (value i for pair i).  A key outside [0, nk) is sorted
// as nk - 1.  offsets, when given, receives the nk + 1 bucket starts
// (offsets[nk] = n).  Seven launches on `st`, no host synchronisation, no
// memset / memcpy nodes (HIP-graph capturable).
hipError_t key_sort_pairs(void *ws, size_t ws_bytes, const int32_t *keys_in, int32_t *keys_out,
                          const int32_t *vals_in, int32_t *vals_out, int64_t n, int32_t nk,
                          const int32_t **offsets, hipStream_t st);

}  // namespace mirec
