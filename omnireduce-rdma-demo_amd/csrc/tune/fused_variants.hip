// fused_variants.hip — tuning harness (not the product): k_scan1f shape variants from the product source,
// timed side by side in one process by tools/tune_fused.py.
#define OMR_NO_CAPI
#include "../omr_kernels.hip"

namespace {
template <int VEC, int W, int LOADS, bool XCD>
void go(const Layout& L, const FusedShape& f, FusedArgs a, hipStream_t st) {
  const unsigned grid = static_cast<unsigned>(static_cast<uint64_t>(L.parts) * L.lanes * f.K);
  const size_t lds = f.nwords * sizeof(uint64_t) + (f.nwords + 1) * sizeof(uint32_t);
  k_scan1f<VEC, W, LOADS, XCD><<<grid, 64 * W, lds, st>>>(a);
}
}  // namespace

extern "C" {
uint32_t omr_sentinel(uint32_t block_size, uint32_t num_lanes) {  // the product's, compiled out by OMR_NO_CAPI
  return (UINT32_MAX / block_size / num_lanes - 1u) * num_lanes * block_size;
}
const char* tune_fused_name(int v) {
  static const char* n[] = {"w8 L16 xcd", "w16 L16 xcd", "w8 L16 noxcd", "w8 L32 xcd", "w8 L8 xcd", "w4 L16 xcd",
                            "w16 L8 xcd"};
  return (v >= 0 && v < 7) ? n[v] : "?";
}
int tune_fused(int v, const float* x, float* out, int32_t* flags, uint32_t* next, void* ws, uint64_t n, uint32_t B,
               uint32_t K, void* stream) {
  Layout L;
  if (make_layout(n, B, 16384 / B, 8, &L)) return -1;
  FusedShape f;
  f.K = K;
  f.S = L.rows_per_part / K;
  f.nwords = (f.S + 63) / 64;
  FusedArgs a;
  a.x = x; a.out = out; a.flags = flags; a.next = next;
  const uint64_t cols = static_cast<uint64_t>(L.parts) * L.lanes;
  a.cnt = static_cast<uint32_t*>(ws);
  a.summary = reinterpret_cast<uint64_t*>(static_cast<char*>(ws) + ((cols * 4 + 15) / 16) * 16);
  a.lanes = L.lanes; a.rpp = L.rows_per_part; a.K = f.K; a.S = f.S; a.block = L.block;
  a.sentinel = omr_sentinel(L.block, L.lanes); a.nwords = f.nwords;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (L.vec == 4) {
    switch (v) {
      case 0: go<4, 8, 16, true>(L, f, a, st); break;
      case 1: go<4, 16, 16, true>(L, f, a, st); break;
      case 2: go<4, 8, 16, false>(L, f, a, st); break;
      case 3: go<4, 8, 32, true>(L, f, a, st); break;
      case 4: go<4, 8, 8, true>(L, f, a, st); break;
      case 5: go<4, 4, 16, true>(L, f, a, st); break;
      case 6: go<4, 16, 8, true>(L, f, a, st); break;
      default: return -3;
    }
    return hipGetLastError() == hipSuccess ? 0 : 1;
  }
  if (L.vec != 1) return -2;
  switch (v) {
    case 0: go<1, 8, 16, true>(L, f, a, st); break;
    case 1: go<1, 16, 16, true>(L, f, a, st); break;
    case 2: go<1, 8, 16, false>(L, f, a, st); break;
    case 3: go<1, 8, 32, true>(L, f, a, st); break;
    case 4: go<1, 8, 8, true>(L, f, a, st); break;
    case 5: go<1, 4, 16, true>(L, f, a, st); break;
    case 6: go<1, 16, 8, true>(L, f, a, st); break;
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
}
