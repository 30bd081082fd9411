// Flash attention kernels instantiated for head dim 32 (templates: attention_impl.h).
#include "attention_impl.h"

namespace apex {

int attn_fwd_d32(const AttnArgs& a, int dt, hipStream_t s) { return attn_fwd_impl<32>(a, dt, s); }

int attn_bwd_d32(const AttnArgs& a, const void* dout, float* delta_ws, void* dk, void* dv, int dt, hipStream_t s) {
  return attn_bwd_impl<32>(a, dout, delta_ws, dk, dv, dt, s);
}

}  // namespace apex
