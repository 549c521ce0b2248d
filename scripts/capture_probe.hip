// capture_probe.hip -- standalone reproduction of launch_step's stream fork/join topology
// (engine.hip) under HIP stream capture, with a trivial kernel in place of the step phases.
//
//   hipcc -O2 --offload-arch=gfx950 -o scripts/capture_probe scripts/capture_probe.hip
//   ./scripts/capture_probe <nsplit> <nclass> <nsub> <piped> [shared_class_streams] [features]
// features (bit mask, engine-like traits added to the trivial kernels):
//   1 warm: run the same launch sequence eagerly (and synchronise) before capturing it
//   2 lds:  kernels take 96 KiB of dynamic LDS (hipFuncSetAttribute beforehand)
//   4 args: kernels take the engine's 7 arguments
//   8 wide: the classify launch is one 1024-thread block
//  16 ovf:  per split a re-solve stream forked after classify (its own event) and joined after
//           the class joins -- round 4's crashing topology (origin -> class streams + re-solve
//           stream, flat forks); its chain is 3 launches (+ the next A when piped)
//  32 replays: replay the instantiated graph 50 times instead of 2
//  64 r4 chain: the re-solve chain as round 4 launched it -- max A, Newton, C, the next A
//           (piped) and a one-thread list-clear kernel (5 launches per substep)
//
// Topology per substep (as launch_step): origin --split_fork--> split streams; on split
// stream k: [A] -> classify -> record fork[k] -> class streams wait -> class chains
// (B [, C, next A]) -> join[k][c] -> split stream waits; after the last substep the split
// streams join the origin.  Every kernel adds 1 to its own counter slot so the replay can
// be checked.  Exit 0 = captured, instantiated, replayed and checked.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 2;                                                                       \
    }                                                                                 \
  } while (0)

__global__ void work(int* slot) {
  if (threadIdx.x == 0 && blockIdx.x == 0) atomicAdd(slot, 1);
}
__global__ void work_lds(int* slot) {
  extern __shared__ int sh[];
  sh[threadIdx.x] = 1;
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) atomicAdd(slot, sh[0]);
}
__global__ void work_args(const int* p, int w0, int w1, int sel, int last, int integ, int* slot) {
  (void)p; (void)w0; (void)w1; (void)sel; (void)last; (void)integ;
  if (threadIdx.x == 0 && blockIdx.x == 0) atomicAdd(slot, 1);
}

// Also built as a shared library (-DPROBE_LIB, scripts/capture_probe_torch.py): probe_run()
// runs the same capture inside a process that has initialised torch, on torch's stream.
static int probe(int nsplit, int nc, int nsub, int piped, int shared, int feat, hipStream_t given);
#ifdef PROBE_LIB
extern "C" int probe_run(int nsplit, int nc, int nsub, int piped, int shared, int feat, void* stream) {
  return probe(nsplit, nc, nsub, piped, shared, feat, (hipStream_t)stream);
}
#else
int main(int argc, char** argv) {
  return probe(argc > 1 ? atoi(argv[1]) : 2, argc > 2 ? atoi(argv[2]) : 1, argc > 3 ? atoi(argv[3]) : 3,
               argc > 4 ? atoi(argv[4]) : 1, argc > 5 ? atoi(argv[5]) : 0, argc > 6 ? atoi(argv[6]) : 0,
               nullptr);
}
#endif
static int probe(int nsplit, int nc, int nsub, int piped, int shared, int feat, hipStream_t given) {
  printf("probe: nsplit=%d nclass=%d nsub=%d piped=%d shared_class_streams=%d features=%d\n", nsplit,
         nc, nsub, piped, shared, feat);
  fflush(stdout);
  hipStream_t origin = given;
  if (!origin) CK(hipStreamCreateWithFlags(&origin, hipStreamNonBlocking));
  std::vector<hipStream_t> split(nsplit);
  std::vector<hipEvent_t> split_join(nsplit);
  hipEvent_t split_fork;
  CK(hipEventCreateWithFlags(&split_fork, hipEventDisableTiming));
  for (int k = 1; k < nsplit; k++) {
    CK(hipStreamCreateWithFlags(&split[k], hipStreamNonBlocking));
    CK(hipEventCreateWithFlags(&split_join[k], hipEventDisableTiming));
  }
  std::vector<std::vector<hipStream_t>> cls(nsplit, std::vector<hipStream_t>(nc));
  std::vector<std::vector<hipEvent_t>> join(nsplit, std::vector<hipEvent_t>(nc));
  std::vector<hipEvent_t> fork(nsplit);
  std::vector<hipStream_t> ovf(nsplit);
  std::vector<hipEvent_t> ovf_fork(nsplit), ovf_join(nsplit);
  for (int k = 0; k < nsplit; k++) {
    CK(hipStreamCreateWithFlags(&ovf[k], hipStreamNonBlocking));
    CK(hipEventCreateWithFlags(&ovf_fork[k], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ovf_join[k], hipEventDisableTiming));
  }
  for (int k = 0; k < nsplit; k++) {
    CK(hipEventCreateWithFlags(&fork[k], hipEventDisableTiming));
    for (int c = 0; c < nc; c++) {
      if (shared && k > 0) cls[k][c] = cls[0][c];
      else CK(hipStreamCreateWithFlags(&cls[k][c], hipStreamNonBlocking));
      CK(hipEventCreateWithFlags(&join[k][c], hipEventDisableTiming));
    }
  }
  const int nslot = 64;
  int* slots;
  CK(hipMalloc(&slots, nslot * sizeof(int)));
  CK(hipMemset(slots, 0, nslot * sizeof(int)));
  CK(hipDeviceSynchronize());
  int expect[nslot] = {};
  const size_t lds = 96 * 1024;
  if (feat & 2) CK(hipFuncSetAttribute((const void*)work_lds, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  bool counting = true;
  auto launch = [&](hipStream_t s, int slot) {
    if (feat & 2)
      hipLaunchKernelGGL(work_lds, dim3(131), dim3(64), lds, s, slots + slot);
    else if (feat & 4)
      hipLaunchKernelGGL(work_args, dim3(131), dim3(64), 0, s, (const int*)slots, 0, 131, 1, 0, 1, slots + slot);
    else
      hipLaunchKernelGGL(work, dim3(4), dim3(64), 0, s, slots + slot);
    if (counting) expect[slot]++;
  };
  auto classify = [&](hipStream_t s, int slot) {
    if (feat & 8) {
      hipLaunchKernelGGL(work, dim3(1), dim3(1024), 0, s, slots + slot);
      if (counting) expect[slot]++;
    } else {
      launch(s, slot);
    }
  };
  for (int k = 0; k < nslot; k++) expect[k] = 0;
  for (int pass = (feat & 1) ? 0 : 1; pass < 2; pass++) {
  counting = pass == 1;
  if (pass == 1) CK(hipStreamBeginCapture(origin, hipStreamCaptureModeGlobal));
  split[0] = origin;
  if (nsplit > 1) {
    CK(hipEventRecord(split_fork, origin));
    for (int k = 1; k < nsplit; k++) CK(hipStreamWaitEvent(split[k], split_fork, 0));
  }
  for (int sub = 0; sub < nsub; sub++) {
    const int last = sub == nsub - 1;
    for (int k = 0; k < nsplit; k++) {
      hipStream_t st = split[k];
      const int base = 8 * k;
      if (!(nc > 0 && piped) || sub == 0) launch(st, base + 0);  // A
      if (nc > 0) {
        classify(st, base + 1);
        if (feat & 16) {
          CK(hipEventRecord(ovf_fork[k], st));
          CK(hipStreamWaitEvent(ovf[k], ovf_fork[k], 0));
          launch(ovf[k], 40 + 4 * k);      // max-carve A
          launch(ovf[k], 40 + 4 * k + 1);  // latency Newton
          launch(ovf[k], 40 + 4 * k + 2);  // C
          if (piped && !last) launch(ovf[k], 40 + 4 * k + 3);  // next A
          if (feat & 64) {  // round 4's list clear: a one-thread kernel
            hipLaunchKernelGGL(work, dim3(1), dim3(1), 0, ovf[k], slots + 60 + k);
            if (counting) expect[60 + k]++;
          }
        }
        CK(hipEventRecord(fork[k], st));
        for (int c = 0; c < nc; c++) {
          CK(hipStreamWaitEvent(cls[k][c], fork[k], 0));
          launch(cls[k][c], base + 2 + c);  // B of class c
          if (piped) {
            launch(cls[k][c], base + 4);  // C
            if (!last) launch(cls[k][c], base + 5);  // next A
          }
        }
        launch(st, base + 6);  // B of the smallest class
        if (piped) {
          launch(st, base + 4);
          if (!last) launch(st, base + 5);
        }
        for (int c = 0; c < nc; c++) {
          CK(hipEventRecord(join[k][c], cls[k][c]));
          CK(hipStreamWaitEvent(st, join[k][c], 0));
        }
        if (feat & 16) {
          CK(hipEventRecord(ovf_join[k], ovf[k]));
          CK(hipStreamWaitEvent(st, ovf_join[k], 0));
        }
        if (piped) continue;
      } else {
        launch(st, base + 6);
      }
      launch(st, base + 7);  // C
    }
  }
  for (int k = 1; k < nsplit; k++) {
    CK(hipEventRecord(split_join[k], split[k]));
    CK(hipStreamWaitEvent(origin, split_join[k], 0));
  }
  if (pass == 0) {  // the eager warm-up run
    CK(hipStreamSynchronize(origin));
    CK(hipDeviceSynchronize());
    CK(hipMemset(slots, 0, nslot * sizeof(int)));
    CK(hipDeviceSynchronize());
    printf("eager pass ok\n");
    fflush(stdout);
  }
  }
  hipGraph_t graph;
  printf("end capture\n");
  fflush(stdout);
  CK(hipStreamEndCapture(origin, &graph));
  size_t nn = 0;
  CK(hipGraphGetNodes(graph, nullptr, &nn));
  printf("captured %zu nodes; instantiate\n", nn);
  fflush(stdout);
  hipGraphExec_t exec;
  CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  printf("launch\n");
  fflush(stdout);
  const int nrep = (feat & 32) ? 50 : 2;
  for (int r = 0; r < nrep; r++) {
    CK(hipGraphLaunch(exec, origin));
    if (r % 10 == 9) {
      CK(hipStreamSynchronize(origin));
      printf("replay %d ok\n", r + 1);
      fflush(stdout);
    }
  }
  CK(hipStreamSynchronize(origin));
  int got[nslot];
  CK(hipMemcpy(got, slots, sizeof(got), hipMemcpyDeviceToHost));
  for (int k = 0; k < nslot; k++)
    if (got[k] != nrep * expect[k]) {
      printf("slot %d: %d != %d\n", k, got[k], nrep * expect[k]);
      return 1;
    }
  printf("ok\n");
  return 0;
}
