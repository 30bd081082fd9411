// Multi-tensor "plan" metadata (device resident).
//
// MI355X-first replacement for the reference's per-parameter host-synced loops
// (apex/amp/scaler.py:6-18, apex/fp16_utils/loss_scaler.py:84-110,
// apex/fp16_utils/fp16util.py:93-129): a tensor list is described ONCE by a
// device-resident table (pointers, sizes, chunk map). Every fused op then runs as
// a single launch over all chunks of all tensors, with no kernel-argument size
// limit (the CUDA design re-launches every ~110 tensors) and no host sync.
#pragma once
#include <stdint.h>

namespace apex {

constexpr int kMaxLists = 6;
constexpr int kChunkShift = 40;  // chunk entry = (tensor << 40) | chunk_index_in_tensor

struct MTMeta {
  int ntensors;
  int nchunks;
  int nlists;
  int chunk_size;        // elements per chunk (multiple of 8)
  int aligned;           // all pointers 16-byte aligned -> vector path allowed
  const int64_t* ptrs;   // [nlists][ntensors] raw addresses
  const int64_t* numel;  // [ntensors]
  const int64_t* chunks; // [nchunks]
  const int64_t* chunk_off;  // [ntensors + 1] first chunk of each tensor

  __host__ __device__ inline void* ptr(int l, int t) const {
    return reinterpret_cast<void*>(ptrs[l * ntensors + t]);
  }
};

// Host-side layout of the packed int64 meta buffer: ptrs | numel | chunk_off | chunks
inline int64_t mt_meta_words(int nlists, int ntensors, int nchunks) {
  return (int64_t)nlists * ntensors + ntensors + (ntensors + 1) + nchunks;
}

inline MTMeta mt_meta_view(const int64_t* dev, int nlists, int ntensors, int nchunks,
                           int chunk_size, int aligned) {
  MTMeta m;
  m.ntensors = ntensors;
  m.nchunks = nchunks;
  m.nlists = nlists;
  m.chunk_size = chunk_size;
  m.aligned = aligned;
  m.ptrs = dev;
  m.numel = dev + (int64_t)nlists * ntensors;
  m.chunk_off = m.numel + ntensors;
  m.chunks = m.chunk_off + ntensors + 1;
  return m;
}

}  // namespace apex
