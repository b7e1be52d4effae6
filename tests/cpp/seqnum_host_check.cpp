// TEST ONLY: the device JSON evaluator of csrc/seqnum.hpp compiled for the host, so the CPU test
// suite can run its logic against the oracle (tests/test_oracle_seqnum.py).  The product path
// runs it only as the sbe_seqnum_kernel launch on the GPU.
#include <cstdint>

#include "../../include/sbecodec.h"

#define SEQNUM_HOST_CHECK 1
#define __device__
#define __forceinline__ inline
#define __constant__ static
namespace {
#include "../../aeron-cluster-client-cpp_amd/csrc/seqnum.hpp"
}

extern "C" uint64_t seqnum_host_eval(const uint8_t* p, uint32_t n) { return json_seq_eval(p, n); }
