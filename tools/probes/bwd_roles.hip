// Timing probe (tools/bwd_roles_probe.py): k_bwd_all with whole block ranges
// ("roles") left out of the grid.  Built into its own .so next to this file;
// the shipped library and its kernels are unchanged (the role ranges are
// just block-count arguments of the same kernel).  Numerics of a masked
// launch are meaningless; timing only.
#include "../../pytorch_operator_1_amd/csrc/kernels/mnist_kernels.hip"

// mask bits: 1 conv2 bias (C), 2 fc2/bias reductions (F), 4 conv2 wgrad (A),
// 8 conv2 dgrad + conv1 wgrad (B), 16 dW1 (D); 32 (with 8): B without the
// fused conv1 wgrad
extern "C" __attribute__((visibility("default"))) int probe_bwd_all(
    const float* g2, const uint8_t* code2, const float* a1p, const float* w2f, const float* x, const uint8_t* code1,
    const float* dh1, const float* a2p, const float* h1, const float* dl, float* p, float* g, float* m,
    long long off_fc2w, long long off_fc2b, long long off_fc1w, long long off_fc1b, long long off_c2w,
    long long off_c2b, long long off_c1w, long long off_c1b, int* ctr, long long* bidx, long long nbatches,
    int* pending, int B, const float* lr, float* c1rep, int nrep, int rep_stride, int mask, hipStream_t s) {
  BwdAllArgs A;
  A.g2 = g2; A.code2 = code2; A.a1p = a1p; A.w2f = w2f; A.x = x; A.code1 = code1;
  A.gw1 = g + off_c1w; A.gb1 = g + off_c1b;
  A.p2w = p + off_c2w; A.g2w = g + off_c2w; A.m2w = m + off_c2w; A.ctr = ctr;
  A.p2b = p + off_c2b; A.m2b = m + off_c2b;
  A.dh1 = dh1; A.a2p = a2p; A.h1 = h1; A.dl = dl;
  A.p1w = p + off_fc1w; A.m1w = m + off_fc1w;
  A.p1b = p + off_fc1b; A.m1b = m + off_fc1b;
  A.pfw = p + off_fc2w; A.mfw = m + off_fc2w;
  A.pfb = p + off_fc2b; A.mfb = m + off_fc2b;
  A.a = sgd_args(lr, 0.5f, 0.f, 1.f, 0);
  A.c1rep = c1rep; A.nrep = nrep; A.rep_stride = rep_stride; A.bias_off = (int)(off_c1b - off_c1w);
  A.grads_only = 0;
  A.g2b = g + off_c2b; A.g1w = g + off_fc1w; A.g1b = g + off_fc1b; A.gfw = g + off_fc2w; A.gfb = g + off_fc2b;
  A.bidx = bidx; A.nbatches = nbatches; A.pending = pending; A.B = B;
  A.nC = (mask & 1) ? (C2 + 3) / 4 : 0;
  A.nF = (mask & 2) ? (((NCLS + 15) / 16) * ((F1OUT + 15) / 16) + 3) / 4 + 9 : 0;
  A.nA = (mask & 4) ? ((B + BWD_WCHUNK - 1) / BWD_WCHUNK) * (32 / BWD_WNTW) : 0;
  A.nB = (mask & 8) ? B * B2_ICG : 0;
  if (mask & 32) {  // dgrad blocks without the fused conv1 wgrad
    A.gw1 = nullptr;
    A.nrep = 1;
  }
  A.dpair = bwd_dpair();
  A.nD = (mask & 16) ? bwd_n_dw1_blocks(A.dpair) : 0;
  A.wpart = nullptr;
  A.hz = nullptr;
  A.nz = 0;
  const size_t ldsA = wgrad_lds_floats<BWD_WCHUNK, BWD_WNTW>() * sizeof(float);
  const size_t ldsB = B2_LDS_FLOATS * sizeof(float);
  const size_t lds = ldsA > ldsB ? ldsA : ldsB;
  const int nblk = A.nA + A.nB + A.nC + A.nD + A.nF;
  if (nblk == 0) return 0;
  hipLaunchKernelGGL(HIP_KERNEL_NAME(k_bwd_all<BWD_WCHUNK, BWD_WNTW>), dim3(nblk), dim3(256), lds, s, A);
  return (int)hipGetLastError();
}

// Resident k_bwd_all blocks per CU as the runtime computes it (registers,
// LDS of the launch's dynamic size, waves).
extern "C" __attribute__((visibility("default"))) int probe_bwd_all_occupancy() {
  const size_t ldsA = wgrad_lds_floats<BWD_WCHUNK, BWD_WNTW>() * sizeof(float);
  const size_t ldsB = B2_LDS_FLOATS * sizeof(float);
  int n = -1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_bwd_all<BWD_WCHUNK, BWD_WNTW>, 256,
                                                   ldsA > ldsB ? ldsA : ldsB) != hipSuccess)
    return -1;
  return n;
}
