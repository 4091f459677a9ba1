// ops_fast.hip -- gfx950 specialisations of the hot-path operators.
// (round-1 bootstrap: no specialisation registered yet; every shape takes
// the generic kernels of ops_generic.hip)
#include "common.hpp"
#include "ops.hpp"

namespace srcnn {
namespace fast {

int try_conv_fwd(const float*, float*, const float*, const float*, uint32_t, uint32_t, uint32_t,
                 uint32_t, uint32_t, int, uint32_t, hipStream_t) {
  return 0;
}

int try_conv_delta(const float*, const float*, float*, const float*, uint32_t, uint32_t,
                   uint32_t, uint32_t, uint32_t, uint32_t, hipStream_t) {
  return 0;
}

size_t grad_workspace_bytes(uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t) {
  return 0;
}

int try_conv_grad_acc(const float*, const float*, float*, float*, uint32_t, uint32_t, uint32_t,
                      uint32_t, uint32_t, uint32_t, void*, size_t, hipStream_t) {
  return 0;
}

}  // namespace fast
}  // namespace srcnn
