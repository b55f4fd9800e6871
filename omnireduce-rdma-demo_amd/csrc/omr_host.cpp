// omr_host.cpp — host-resident worker round: the gradient starts and ends in (pinned) host memory, as the
// reference's registered region does (common.cc:873-914; the worker fills res->buf, client.cc:401-421, and gets
// the aggregated blocks back in place, client.cc:89).  The tensor is streamed H2D in row chunks on one HIP
// stream, each landed chunk is scanned + aggregated in place on a second (omr_scan_sum_rows_f32), and the chunk
// goes back D2H on a third, so PCIe reads, HBM work and PCIe writes overlap; the next-offset chains run once all
// rows are scanned.  The zero-copy variant skips the staging: the single-pass kernel reads and writes the pinned
// buffer itself over PCIe (tools/bench_host.py: 52 GB/s vs 47 GB/s staged at 4 GiB, 52 vs 40 at 256 MiB).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <vector>

#include "omr.h"

struct omr_host_plan {
  uint64_t n = 0, rows = 0, nb = 0, chunk_rows = 0, nchunks = 0;
  uint32_t block = 0, lanes = 0, parts = 0;
  float* d_buf = nullptr;
  int32_t* d_flags = nullptr;
  uint64_t* d_masks = nullptr;
  uint32_t* d_next = nullptr;
  void* d_ws = nullptr;  // single-pass kernel workspace (zero-copy path), zeroed once, left zeroed by every launch
  size_t ws_bytes = 0;
  hipStream_t s_in = nullptr, s_cmp = nullptr, s_out = nullptr;
  std::vector<hipEvent_t> ev_in, ev_cmp;
  hipEvent_t ev_done_out = nullptr;
};

namespace {

thread_local char g_host_err[256];

int herr(hipError_t e, const char* what) {
  if (e == hipSuccess) return 0;
  snprintf(g_host_err, sizeof(g_host_err), "%s: %s", what, hipGetErrorString(e));
  return static_cast<int>(e);
}

#define OMR_HIP(call)                                  \
  do {                                                 \
    if (int _rc = herr((call), #call)) return _rc;     \
  } while (0)

// A library call failed partway through a pipelined round: copies already queued keep running into the host
// buffer and the device buffer, so let them drain before returning, and report the library's message here.
int fail_drain(omr_host_plan* p, int rc, const char* what) {
  snprintf(g_host_err, sizeof(g_host_err), "%s: %s", what, omr_last_error());
  for (hipStream_t s : {p->s_in, p->s_cmp, p->s_out})
    if (s) (void)hipStreamSynchronize(s);
  return rc;
}

}  // namespace

extern "C" {

const char* omr_host_last_error(void) { return g_host_err; }

int omr_host_register(void* ptr, size_t bytes) {
  return herr(hipHostRegister(ptr, bytes, hipHostRegisterDefault), "hipHostRegister");
}

int omr_host_unregister(void* ptr) { return herr(hipHostUnregister(ptr), "hipHostUnregister"); }

int omr_host_plan_destroy(omr_host_plan* p) {
  if (p == nullptr) return 0;
  for (hipEvent_t e : p->ev_in) (void)hipEventDestroy(e);
  for (hipEvent_t e : p->ev_cmp) (void)hipEventDestroy(e);
  if (p->ev_done_out) (void)hipEventDestroy(p->ev_done_out);
  if (p->s_in) (void)hipStreamDestroy(p->s_in);
  if (p->s_cmp) (void)hipStreamDestroy(p->s_cmp);
  if (p->s_out) (void)hipStreamDestroy(p->s_out);
  (void)hipFree(p->d_buf);
  (void)hipFree(p->d_flags);
  (void)hipFree(p->d_masks);
  (void)hipFree(p->d_next);
  (void)hipFree(p->d_ws);
  delete p;
  return 0;
}

int omr_host_plan_create(uint64_t n, uint32_t block_size, uint32_t num_lanes, uint32_t num_parts,
                         uint64_t chunk_rows, omr_host_plan** out) {
  if (out == nullptr) return OMR_EINVAL;
  *out = nullptr;
  if (int rc = omr_layout_check(n, block_size, num_lanes, num_parts)) return rc;
  auto* p = new omr_host_plan();
  p->n = n;
  p->block = block_size;
  p->lanes = num_lanes;
  p->parts = num_parts;
  p->nb = n / block_size;
  p->rows = p->nb / num_lanes;
  p->chunk_rows = chunk_rows == 0 ? 512 : chunk_rows;
  if (p->chunk_rows > p->rows) p->chunk_rows = p->rows;
  p->nchunks = (p->rows + p->chunk_rows - 1) / p->chunk_rows;
  int rc = 0;
  auto H = [&](hipError_t e, const char* w) {
    if (rc == 0) rc = herr(e, w);
  };
  H(hipMalloc(&p->d_buf, n * sizeof(float)), "hipMalloc buf");
  H(hipMalloc(&p->d_flags, p->nb * sizeof(int32_t)), "hipMalloc flags");
  H(hipMalloc(&p->d_masks, p->rows * sizeof(uint64_t)), "hipMalloc masks");
  H(hipMalloc(&p->d_next, p->nb * sizeof(uint32_t)), "hipMalloc next");
  p->ws_bytes = omr_scan_workspace_bytes(n, block_size, num_lanes, num_parts);
  if (p->ws_bytes) {
    H(hipMalloc(&p->d_ws, p->ws_bytes), "hipMalloc workspace");
    H(hipMemset(p->d_ws, 0, p->ws_bytes), "hipMemset workspace");
  }
  H(hipStreamCreateWithFlags(&p->s_in, hipStreamNonBlocking), "stream");
  H(hipStreamCreateWithFlags(&p->s_cmp, hipStreamNonBlocking), "stream");
  H(hipStreamCreateWithFlags(&p->s_out, hipStreamNonBlocking), "stream");
  p->ev_in.resize(p->nchunks, nullptr);
  p->ev_cmp.resize(p->nchunks, nullptr);
  for (uint64_t k = 0; k < p->nchunks && rc == 0; ++k) {
    H(hipEventCreateWithFlags(&p->ev_in[k], hipEventDisableTiming), "event");
    H(hipEventCreateWithFlags(&p->ev_cmp[k], hipEventDisableTiming), "event");
  }
  H(hipEventCreateWithFlags(&p->ev_done_out, hipEventDisableTiming), "event");
  if (rc != 0) {
    omr_host_plan_destroy(p);
    return rc;
  }
  *out = p;
  return 0;
}

int omr_host_scan_sum_f32(omr_host_plan* p, float* host_buf, int32_t* host_flags, uint32_t* host_next,
                          double* seconds) {
  if (p == nullptr || host_buf == nullptr) {
    snprintf(g_host_err, sizeof(g_host_err), "host_scan_sum: NULL plan or buffer");
    return OMR_EINVAL;
  }
  const auto t0 = std::chrono::steady_clock::now();
  const uint64_t row_floats = static_cast<uint64_t>(p->lanes) * p->block;
  // Write-back: with a device mapping of the pinned buffer, the scan stores its aggregated blocks (non-zero blocks
  // and lane heads, the ones the reference's worker gets back: client.cc:89) straight into it, beside the copy
  // engine's H2D of the next chunk; every other block is zero and unchanged.  Without one (or with
  // OMR_HOST_STAGED_D2H set) each chunk is copied back whole.
  float* hdev = nullptr;
  {
    void* d = nullptr;
    if (getenv("OMR_HOST_STAGED_D2H") == nullptr && hipHostGetDevicePointer(&d, host_buf, 0) == hipSuccess && d)
      hdev = static_cast<float*>(d);
    else
      (void)hipGetLastError();
  }
  for (uint64_t k = 0; k < p->nchunks; ++k) {
    const uint64_t r0 = k * p->chunk_rows;
    const uint64_t r1 = (r0 + p->chunk_rows < p->rows) ? r0 + p->chunk_rows : p->rows;
    const uint64_t off = r0 * row_floats;
    const size_t bytes = (r1 - r0) * row_floats * sizeof(float);
    OMR_HIP(hipMemcpyAsync(p->d_buf + off, host_buf + off, bytes, hipMemcpyHostToDevice, p->s_in));
    OMR_HIP(hipEventRecord(p->ev_in[k], p->s_in));
    OMR_HIP(hipStreamWaitEvent(p->s_cmp, p->ev_in[k], 0));
    if (int rc = omr_scan_sum_rows_f32(p->d_buf, p->n, p->block, p->lanes, p->parts, r0, r1, p->d_flags,
                                       p->d_masks, hdev ? hdev : p->d_buf, p->s_cmp))
      return fail_drain(p, rc, "omr_scan_sum_rows_f32");
    if (hdev) continue;
    OMR_HIP(hipEventRecord(p->ev_cmp[k], p->s_cmp));
    OMR_HIP(hipStreamWaitEvent(p->s_out, p->ev_cmp[k], 0));
    OMR_HIP(hipMemcpyAsync(host_buf + off, p->d_buf + off, bytes, hipMemcpyDeviceToHost, p->s_out));
  }
  if (int rc = omr_next_offsets(p->d_masks, 1, p->n, p->block, p->lanes, p->parts, p->d_next, p->s_cmp))
    return fail_drain(p, rc, "omr_next_offsets");
  if (host_flags != nullptr)
    OMR_HIP(hipMemcpyAsync(host_flags, p->d_flags, p->nb * sizeof(int32_t), hipMemcpyDeviceToHost, p->s_cmp));
  if (host_next != nullptr)
    OMR_HIP(hipMemcpyAsync(host_next, p->d_next, p->nb * sizeof(uint32_t), hipMemcpyDeviceToHost, p->s_cmp));
  OMR_HIP(hipStreamSynchronize(p->s_out));
  OMR_HIP(hipStreamSynchronize(p->s_cmp));
  if (seconds != nullptr)
    *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return 0;
}

int omr_host_scan_sum_zero_copy_f32(omr_host_plan* p, float* host_buf, int32_t* host_flags, uint32_t* host_next,
                                    double* seconds) {
  if (p == nullptr || host_buf == nullptr) {
    snprintf(g_host_err, sizeof(g_host_err), "host_scan_sum_zero_copy: NULL plan or buffer");
    return OMR_EINVAL;
  }
  const auto t0 = std::chrono::steady_clock::now();
  // the buffer's address in the GPU's space (pinned memory only: pageable memory has none)
  void* dev = nullptr;
  if (hipHostGetDevicePointer(&dev, host_buf, 0) != hipSuccess || dev == nullptr) {
    (void)hipGetLastError();
    snprintf(g_host_err, sizeof(g_host_err), "zero-copy: host_buf is not pinned (omr_host_register / hipHostMalloc)");
    return OMR_EINVAL;
  }
  float* buf = static_cast<float*>(dev);
  if (int rc = omr_scan_sum_fused_f32(buf, p->n, p->block, p->lanes, p->parts, p->d_flags, p->d_next, buf, p->d_ws,
                                      p->ws_bytes, p->s_cmp)) {
    snprintf(g_host_err, sizeof(g_host_err), "omr_scan_sum_fused_f32: %s", omr_last_error());
    return rc;
  }
  if (host_flags != nullptr)
    OMR_HIP(hipMemcpyAsync(host_flags, p->d_flags, p->nb * sizeof(int32_t), hipMemcpyDeviceToHost, p->s_cmp));
  if (host_next != nullptr)
    OMR_HIP(hipMemcpyAsync(host_next, p->d_next, p->nb * sizeof(uint32_t), hipMemcpyDeviceToHost, p->s_cmp));
  OMR_HIP(hipStreamSynchronize(p->s_cmp));
  if (seconds != nullptr)
    *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return 0;
}

}  // extern "C"
