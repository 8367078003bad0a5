// Timed-window markers for kernel traces: bench.py launches lk_window_mark_kernel(1) right
// after the barrier + synchronize that opens its timed window and (2) right before the one that
// closes it (LK_TRACE_WINDOW=1), so scripts/summarize_trace.py bounds a rocprofv3 kernel trace to
// exactly the timed steps -- no warm-up, no drain -- without roctx / marker tracing.
#include "common.h"
#include "kernels.h"

namespace {
__global__ __launch_bounds__(64) void lk_window_mark_kernel(int id, int* sink) {
  if (sink && threadIdx.x == 0) sink[0] = id;  // one vector store: never optimised away
}
int* g_sink = nullptr;
}  // namespace

int lk_window_mark(int id, hipStream_t st) {
  if (!g_sink && hipMalloc(&g_sink, sizeof(int)) != hipSuccess) return -1;
  lk_window_mark_kernel<<<1, 64, 0, st>>>(id, g_sink);
  return 0;
}

// Loud-failure probe (tests/test_kernels_gpu.py): a launch the runtime must reject before any
// wave runs (2048 threads per workgroup, above the 1024 limit), checked like every launcher.
int lk_debug_invalid_launch(hipStream_t st) {
  lk_window_mark_kernel<<<1, 2048, 0, st>>>(0, nullptr);
  LK_CHECK_LAUNCH();
  return 0;
}
