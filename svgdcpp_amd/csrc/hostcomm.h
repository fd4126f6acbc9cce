// Host shared-memory collectives for multi-rank rehearsal on one GPU
// (see hostcomm.cpp).  All return 0 on success.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace svgd_amd {
struct HostComm;
int hostcomm_create(HostComm **out, const char *name, int world, int rank, size_t slot_bytes);
void hostcomm_destroy(HostComm *c);
int hostcomm_allgather(HostComm *c, char *dbuf, size_t count_bytes, hipStream_t stream);
int hostcomm_allreduce_u32(HostComm *c, uint32_t *dbuf, size_t cnt, hipStream_t stream);
int hostcomm_allreduce_f64(HostComm *c, double *dbuf, size_t cnt, hipStream_t stream);
int hostcomm_exchange_f64(HostComm *c, double *dsend, size_t n, size_t w, const int64_t *send,
                          double *drecv, size_t recv_rows, const int64_t *recv, int64_t own0, int64_t own1,
                          hipStream_t stream);
int hostcomm_allreduce_u64(HostComm *c, unsigned long long *dbuf, size_t cnt, hipStream_t stream);
} // namespace svgd_amd
