// fused_variants.hip — tuning harness (not the product): k_scan1f shapes (waves per workgroup, loads in flight)
// and timing-only ablations (ABL bit 0: no data stores, bit 1: no flag/next stores) from the product source,
// timed side by side by tools/tune_fused.py.
#define OMR_NO_CAPI
#include "../omr_kernels.hip"

namespace {
template <int VEC, int W, int LOADS, int ABL>
void go_f(const Layout& L, const FusedShape& f, FusedArgs a, hipStream_t st) {
  const unsigned grid = static_cast<unsigned>(static_cast<uint64_t>(L.parts) * L.lanes * f.K);
  k_scan1f<VEC, W, LOADS, ABL><<<grid, 64 * W, 0, st>>>(a);
}

struct Variant {
  const char* name;
  bool checked;  // produces the full outputs (ablations do not)
  void (*v1)(const Layout&, const FusedShape&, FusedArgs, hipStream_t);
  void (*v4)(const Layout&, const FusedShape&, FusedArgs, hipStream_t);
};

#define VF(W, LD, A) go_f<1, W, LD, A>, go_f<4, W, LD, A>
const Variant kVariants[] = {
    {"w16 L16", true, VF(16, 16, 0)},
    {"w16 L8", true, VF(16, 8, 0)},
    {"w8 L16", true, VF(8, 16, 0)},
    {"w8 L8", true, VF(8, 8, 0)},
    {"w4 L16", true, VF(4, 16, 0)},
    {"w16 L32", true, VF(16, 32, 0)},
    {"w16 L16 -data", false, VF(16, 16, 1)},
    {"w16 L16 -meta", false, VF(16, 16, 2)},
    {"w16 L16 -data-meta", false, VF(16, 16, 3)},
};
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);
}  // namespace

extern "C" {
uint32_t omr_sentinel(uint32_t block_size, uint32_t num_lanes) {  // the product's, compiled out by OMR_NO_CAPI
  return (UINT32_MAX / block_size / num_lanes - 1u) * num_lanes * block_size;
}
int tune_fused_count(void) { return kNumVariants; }
const char* tune_fused_name(int v) { return (v >= 0 && v < kNumVariants) ? kVariants[v].name : "?"; }
int tune_fused_checked(int v) { return (v >= 0 && v < kNumVariants) ? kVariants[v].checked : 0; }
int tune_fused(int v, const float* x, float* out, int32_t* flags, uint32_t* next, void* ws, uint64_t n, uint32_t B,
               uint32_t K, void* stream) {
  Layout L;
  if (v < 0 || v >= kNumVariants) return -3;
  if (make_layout(n, B, 16384 / B, 8, &L)) return -1;
  FusedShape f;
  f.K = K;
  f.S = L.rows_per_part / K;
  FusedArgs a;
  a.x = x; a.out = out; a.flags = flags; a.next = next;
  const uint64_t cols = static_cast<uint64_t>(L.parts) * L.lanes;
  a.cnt = static_cast<uint32_t*>(ws);
  a.summary = reinterpret_cast<uint64_t*>(static_cast<char*>(ws) + ((cols * 4 + 15) / 16) * 16);
  a.lanes = L.lanes; a.rpp = L.rows_per_part; a.K = f.K; a.S = f.S; a.block = L.block;
  a.sentinel = omr_sentinel(L.block, L.lanes);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (L.vec == 4) kVariants[v].v4(L, f, a, st);
  else if (L.vec == 1) kVariants[v].v1(L, f, a, st);
  else return -2;
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
}
