// One-time kernel attribute setup (dynamic LDS > 64 KiB for head_dim 256).
#include "launchers.h"

namespace drtc {
int configure_kernels() {
  int e = configure_decode();
  if (e) return e;
  e = configure_prefill();
  if (e) return e;
  e = configure_moe();
  if (e) return e;
  e = configure_gemm_w4();
  if (e) return e;
  return configure_gemm_xd();
}
}  // namespace drtc
