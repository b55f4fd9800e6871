// worker_partition.cpp — INTEGRATION.md's worker recipe, compiled and run as the reference runs its workers
// (test program, not the product).  A worker process holds its gradient in a posix_memalign'd host region, as
// resources_create does (common.cc:873-914), filled by the reference generator itself (client.cc:396-421:
// srand(id + 1), glibc rand(), 0.01f blocks).  NUM_THREADS std::threads, one per partition as
// process_per_thread (client.cc:168, started at :384-392), each on its own HIP stream, run exactly the recipe:
// H2D of the partition, omr_scan_partition_f32, D2H of the partition's next offsets and flags.  Then every block's
// next offset is compared with the oracle's literal restatement of find_next_nonzero_block (client.cc:19-31,
// oracle/omr_oracle.c), called as the reference calls it (off + BLOCK_SIZE * NUM_BLOCKS), and every flag with the
// generator's bitmap.  A second pass writes the aggregated (m = 1) blocks in place and checks them bit for bit.
//   usage: worker_partition [-n floats] [-b block_size] [-r density] [-i worker_id]     exit 0 = all equal
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "omr.h"
#include "omr_oracle.h"

#define HIPCK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                      \
    }                                                                               \
  } while (0)

int main(int argc, char** argv) {
  uint64_t DATA_SIZE = 16ull << 20;  // floats (common.h:40 style); 64 MiB by default
  uint32_t BLOCK_SIZE = 256, id = 0;
  double ratio = 0.095;
  const uint32_t NUM_THREADS = 8;  // common.h:29
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!strcmp(argv[i], "-n")) DATA_SIZE = strtoull(argv[i + 1], nullptr, 0);
    else if (!strcmp(argv[i], "-b")) BLOCK_SIZE = static_cast<uint32_t>(strtoul(argv[i + 1], nullptr, 0));
    else if (!strcmp(argv[i], "-r")) ratio = atof(argv[i + 1]);
    else if (!strcmp(argv[i], "-i")) id = static_cast<uint32_t>(strtoul(argv[i + 1], nullptr, 0));
  }
  const uint32_t NUM_BLOCKS = omr_num_lanes(BLOCK_SIZE);
  const uint64_t DATA_SIZE_PER_THREAD = DATA_SIZE / NUM_THREADS;
  if (omr_layout_check(DATA_SIZE, BLOCK_SIZE, NUM_BLOCKS, NUM_THREADS)) {
    fprintf(stderr, "layout: %s\n", omr_last_error());
    return 2;
  }
  const uint64_t nb = DATA_SIZE / BLOCK_SIZE;

  // the worker's region and bitmap, generated as client.cc:396-421 does (the real glibc rand)
  float* buf = nullptr;
  int32_t* bitmap = nullptr;
  if (posix_memalign(reinterpret_cast<void**>(&buf), 4096, DATA_SIZE * 4) ||
      posix_memalign(reinterpret_cast<void**>(&bitmap), 4096, nb * 4))
    return 2;
  srand(id + 1);
  for (uint64_t i = 0; i < nb; ++i) {
    bitmap[i] = (rand() % 100 / static_cast<double>(101) < ratio) ? 1 : 0;
    const float v = bitmap[i] ? 0.01f : 0.0f;
    for (uint32_t j = 0; j < BLOCK_SIZE; ++j) buf[i * BLOCK_SIZE + j] = v;
  }

  // the recipe's one-time setup
  float* d_buf;
  int32_t* d_flags;
  uint32_t* d_next;
  void* d_ws;
  HIPCK(hipMalloc(&d_buf, DATA_SIZE * 4));
  HIPCK(hipMalloc(&d_flags, nb * 4));
  HIPCK(hipMalloc(&d_next, nb * 4));
  const size_t ws_bytes = omr_scan_workspace_bytes(DATA_SIZE, BLOCK_SIZE, NUM_BLOCKS, NUM_THREADS);
  HIPCK(hipMalloc(&d_ws, ws_bytes ? ws_bytes : 16));
  HIPCK(hipMemset(d_ws, 0, ws_bytes ? ws_bytes : 16));
  std::vector<uint32_t> next_host(nb, 0);
  std::vector<int32_t> flags_host(nb, -1);
  std::vector<float> back(DATA_SIZE);

  for (int pass = 0; pass < 2; ++pass) {  // pass 1: also the aggregated blocks in place (out = d_buf)
    std::vector<int> rc(NUM_THREADS, 0);
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < NUM_THREADS; ++t) {
      th.emplace_back([&, t] {  // process_per_thread (client.cc:168), res->threadId == t
        HIPCK(hipSetDevice(0));
        hipStream_t st;
        HIPCK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        const uint32_t part = t;
        const uint64_t p0 = static_cast<uint64_t>(part) * DATA_SIZE_PER_THREAD, pb0 = p0 / BLOCK_SIZE;
        const uint64_t pnb = DATA_SIZE_PER_THREAD / BLOCK_SIZE;
        HIPCK(hipMemcpyAsync(d_buf + p0, buf + p0, DATA_SIZE_PER_THREAD * 4, hipMemcpyHostToDevice, st));
        if (omr_scan_partition_f32(d_buf, DATA_SIZE, BLOCK_SIZE, NUM_BLOCKS, NUM_THREADS, part, d_flags, d_next,
                                   pass ? d_buf : nullptr, d_ws, ws_bytes, st)) {
          fprintf(stderr, "omr_scan_partition_f32: %s\n", omr_last_error());
          rc[t] = 1;
        }
        HIPCK(hipMemcpyAsync(next_host.data() + pb0, d_next + pb0, pnb * 4, hipMemcpyDeviceToHost, st));
        HIPCK(hipMemcpyAsync(flags_host.data() + pb0, d_flags + pb0, pnb * 4, hipMemcpyDeviceToHost, st));
        if (pass) HIPCK(hipMemcpyAsync(back.data() + p0, d_buf + p0, DATA_SIZE_PER_THREAD * 4, hipMemcpyDeviceToHost, st));
        HIPCK(hipStreamSynchronize(st));
        HIPCK(hipStreamDestroy(st));
      });
    }
    for (auto& x : th) x.join();
    for (int r : rc)
      if (r) return 1;
    // every block: next_host[b] == find_next_nonzero_block(res, b*BLOCK_SIZE + BLOCK_SIZE*NUM_BLOCKS) of its thread
    uint64_t bad_next = 0, bad_flag = 0, bad_out = 0;
    for (uint64_t b = 0; b < nb; ++b) {
      const uint32_t tid = static_cast<uint32_t>(b * BLOCK_SIZE / DATA_SIZE_PER_THREAD);
      const uint32_t off = static_cast<uint32_t>(b * BLOCK_SIZE + static_cast<uint64_t>(BLOCK_SIZE) * NUM_BLOCKS);
      const uint32_t want = orc_find_next_nonzero_block(bitmap, static_cast<uint32_t>(DATA_SIZE_PER_THREAD),
                                                        BLOCK_SIZE, NUM_BLOCKS, tid, off);
      bad_next += next_host[b] != want;
      bad_flag += flags_host[b] != bitmap[b];
    }
    if (pass) bad_out = memcmp(back.data(), buf, DATA_SIZE * 4) != 0;  // 0.0f + x == x for the generator's data
    printf("pass %d (%s): %llu blocks, %u threads: next mismatches %llu, flag mismatches %llu%s\n", pass,
           pass ? "scan + aggregated blocks in place" : "scan", static_cast<unsigned long long>(nb), NUM_THREADS,
           static_cast<unsigned long long>(bad_next), static_cast<unsigned long long>(bad_flag),
           pass ? (bad_out ? ", out DIFFERS" : ", out equal") : "");
    if (bad_next || bad_flag || bad_out) return 1;
  }
  HIPCK(hipFree(d_buf));
  HIPCK(hipFree(d_flags));
  HIPCK(hipFree(d_next));
  HIPCK(hipFree(d_ws));
  free(buf);
  free(bitmap);
  return 0;
}
