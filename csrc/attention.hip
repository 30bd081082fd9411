// Flash attention (NS-05): head-dim dispatch and the dropout-mask debug kernel. The kernel
// templates live in attention_impl.h; attention_d{32,64,128,256}.hip instantiate one head dim
// each so the (many) variants compile in parallel.
#include "attention_impl.h"

namespace apex {

// debug / test: materialise the keep-mask the kernels use (uint8 [B*H, Sq, Sk])
__global__ void attn_dropout_mask_kernel(uint8_t* out, int64_t BH, int Sq, int Sk, uint64_t seed,
                                         uint64_t offset, uint32_t thresh) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;  // one thread per 32 keys
  const int64_t nblk = (Sk + 31) / 32;
  if (idx >= BH * Sq * nblk) return;
  const int64_t blk = idx % nblk, row = idx / nblk;
  const int q = (int)(row % Sq);
  const int64_t bh = row / Sq;
  const uint32_t w = drop_block_bits(seed, offset, thresh, bh, q, blk, Sq);
  for (int k = 0; k < 32; ++k) {
    const int64_t key = blk * 32 + k;
    if (key < Sk) out[row * Sk + key] = (w >> k) & 1;
  }
}

int attn_dropout_mask(uint8_t* out, int64_t BH, int Sq, int Sk, uint64_t seed, uint64_t offset,
                      uint32_t thresh, hipStream_t s) {
  const int64_t n = BH * Sq * ((Sk + 31) / 32);
  hipLaunchKernelGGL(attn_dropout_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     out, BH, Sq, Sk, seed, offset, thresh);
  return (int)hipGetLastError();
}


int attn_fwd(const AttnArgs& a, int dt, hipStream_t s) {
  if (a.B * a.H == 0 || a.Sq == 0) return 0;
  if (a.drop_thresh > 0 && !a.dmask) return -3;
  if (dt == kF32) return attn_fwd_f32(a, s);
  switch (a.D) {
    case 32: return attn_fwd_d32(a, dt, s);
    case 64: return attn_fwd_d64(a, dt, s);
    case 128: return attn_fwd_d128(a, dt, s);
    case 256: return attn_fwd_d256(a, dt, s);
    default: return -1;
  }
}

// Two-kernel backward (key-stationary dK/dV + query-stationary dQ, delta pre-pass) for key ranges
// longer than one 128-key block; APEX_ATTN_BWD_SPLIT=1 also selects it for short ones (A/B knob)
bool attn_bwd_split() {
  static const bool on = [] {
    const char* e = getenv("APEX_ATTN_BWD_SPLIT");
    return e && e[0] == '1';
  }();
  return on;
}
bool attn_bwd_needs_dq_acc(const AttnArgs& a) { return a.Sk > kBwdBK || attn_bwd_split(); }

int attn_bwd(const AttnArgs& a, const void* dout, float* delta_ws, void* dk, void* dv, int dt,
             hipStream_t s) {
  if (a.B * a.H == 0 || a.Sq == 0) return 0;
  if (a.drop_thresh > 0 && !a.dmask) return -3;  // backward needs the forward's dropout bits
  if (dt == kF32) return attn_bwd_f32(a, dout, delta_ws, dk, dv, s);
  switch (a.D) {
    case 32: return attn_bwd_d32(a, dout, delta_ws, dk, dv, dt, s);
    case 64: return attn_bwd_d64(a, dout, delta_ws, dk, dv, dt, s);
    case 128: return attn_bwd_d128(a, dout, delta_ws, dk, dv, dt, s);
    case 256: return attn_bwd_d256(a, dout, delta_ws, dk, dv, dt, s);
    default: return -1;
  }
}

}  // namespace apex
