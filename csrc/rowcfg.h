// Row-per-workgroup launch shape shared by the row-wise norm kernels (norm.hip) and the
// fused all-reduce + RMSNorm of the TP decode step (xgmi_allreduce.hip): both must slice a
// row over threads identically for their results to be bit-identical.
#pragma once

// pick (waves, vectors-per-thread) so that a row is covered with all values in registers
struct RowCfg {
  int nw, maxv;
};
inline RowCfg row_cfg(int H) {
  const int nvec = H / 8;
  int nw = nvec >= 1024 ? 4 : (nvec >= 512 ? 4 : (nvec >= 256 ? 4 : (nvec >= 128 ? 2 : 1)));
  int maxv = (nvec + nw * 64 - 1) / (nw * 64);
  return {nw, maxv};
}

#define ROW_DISPATCH(H, KERNEL_CALL)                                           \
  do {                                                                         \
    RowCfg cfg_ = row_cfg(H);                                                  \
    if (cfg_.nw == 1 && cfg_.maxv == 1) { KERNEL_CALL(1, 1); }                 \
    else if (cfg_.nw == 1 && cfg_.maxv == 2) { KERNEL_CALL(2, 1); }            \
    else if (cfg_.nw == 2 && cfg_.maxv == 1) { KERNEL_CALL(1, 2); }            \
    else if (cfg_.nw == 4 && cfg_.maxv == 1) { KERNEL_CALL(1, 4); }            \
    else if (cfg_.nw == 4 && cfg_.maxv == 2) { KERNEL_CALL(2, 4); }            \
    else if (cfg_.nw == 4 && cfg_.maxv <= 4) { KERNEL_CALL(4, 4); }            \
    else if (cfg_.nw == 4 && cfg_.maxv <= 8) { KERNEL_CALL(8, 4); }            \
    else { return -1; }                                                        \
  } while (0)
