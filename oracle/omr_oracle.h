/* omr_oracle.h — CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY; see omr_oracle.c). */
#ifndef OMR_ORACLE_H
#define OMR_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

uint32_t orc_sentinel(uint32_t B, uint32_t NB);
uint64_t orc_gen_bitmap(uint32_t worker_id, double density, uint64_t nb, int32_t* bitmap);
void orc_fill(const int32_t* bitmap, uint64_t nb, uint32_t B, int mode, uint32_t seed, float* buf);
void orc_flags_from_data(const float* buf, uint64_t nb, uint32_t B, int32_t* flags);
void orc_row_masks(const int32_t* flags, uint64_t nb, uint32_t NB, uint64_t* masks);
void orc_union_flags(const int32_t* flags, uint32_t m, uint64_t nb, int32_t* out);
uint32_t orc_find_next_nonzero_block(const int32_t* flags, uint32_t P, uint32_t B, uint32_t NB, uint32_t tid,
                                     uint32_t next_offset);
void orc_next_offsets(const int32_t* flags, uint64_t n, uint32_t B, uint32_t NB, uint32_t parts,
                      uint32_t* next);
void orc_block_sum(const float* const* bufs, uint32_t m, uint64_t n, uint32_t B, uint32_t NB, uint32_t parts,
                   const int32_t* uflags, float* out);
uint32_t orc_lane_stream(const int32_t* flags, uint64_t n, uint32_t B, uint32_t NB, uint32_t parts, uint32_t tid,
                         uint32_t bid, uint32_t* cur_out, uint32_t* next_out, uint32_t cap);
int orc_msg_simulate(const float* const* bufs, const int32_t* const* flags, uint32_t m, uint64_t n, uint32_t B,
                     uint32_t NB, uint32_t parts, uint32_t rcap, float* wmsg, uint32_t* wimm, float* rmsg,
                     uint32_t* rimm, float* const* outs, uint32_t* rounds);
double orc_cpu_baseline(const float* x, const int32_t* bitmap, uint64_t n, uint32_t B, uint32_t NB,
                        uint32_t parts, uint32_t nthreads, uint32_t variant, int warmups, int rounds,
                        int32_t* flags, uint32_t* next, float* out);
/* Cores the last orc_cpu_baseline run pinned its threads to; returns how many were written to out. */
int orc_cpu_baseline_cores(int* out, int cap);

#ifdef __cplusplus
}
#endif
#endif
