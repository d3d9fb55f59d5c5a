// mailbox_probe.hip — where should the resident server's mailbox live? Measures the host -> device
// -> host ping-pong latency of a one-wave polling kernel for a request word in (a) pinned coherent
// host memory (the r03 design: the device polls over PCIe) and (b) device memory the host writes
// through its mapping (fine-grained / uncached device allocations, if the host can map them);
// the acknowledgement always goes to pinned host memory. Usage: mailbox_probe pinned|fine|uncached
// (one kind per process: if the host cannot touch a device allocation, the host store faults and
// ends that process only, with no kernel running).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                               \
    }                                                                         \
  } while (0)

// req[0] = sequence number from the host (0 = none yet, 0xffffffff = stop); ack[0] = last seen
__global__ void pong(const uint32_t* req, uint32_t* ack, uint64_t max_ticks) {
  uint32_t seen = 0;
  const uint64_t t0 = wall_clock64();
  for (;;) {
    const uint32_t v = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v == 0xffffffffu || wall_clock64() - t0 > max_ticks) break;
    if (v != seen) {
      seen = v;
      if (threadIdx.x == 0) __hip_atomic_store(ack, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

static int pingpong(const char* name, uint32_t* req_host_view, const uint32_t* req_dev_view, uint32_t* ack_host,
                    uint32_t* ack_dev, int khz) {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  __atomic_store_n(req_host_view, 0u, __ATOMIC_SEQ_CST);
  __atomic_store_n(ack_host, 0u, __ATOMIC_SEQ_CST);
  hipLaunchKernelGGL(pong, dim3(1), dim3(64), 0, s, req_dev_view, ack_dev, (uint64_t)khz * 1000ull * 20);  // 20 s cap
  CK(hipGetLastError());
  std::vector<double> us;
  for (uint32_t k = 1; k <= 3000; ++k) {
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(req_host_view, k, __ATOMIC_SEQ_CST);
    while (__atomic_load_n(ack_host, __ATOMIC_ACQUIRE) != k) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
        std::printf("%s: no ack for request %u\n", name, k);
        __atomic_store_n(req_host_view, 0xffffffffu, __ATOMIC_SEQ_CST);
        (void)hipStreamSynchronize(s);
        return 1;
      }
    }
    us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  __atomic_store_n(req_host_view, 0xffffffffu, __ATOMIC_SEQ_CST);
  CK(hipStreamSynchronize(s));
  CK(hipStreamDestroy(s));
  std::sort(us.begin() + 200, us.end());
  const size_t n = us.size() - 200;
  std::printf("%-34s round trip median %.2f us, p10 %.2f, p99 %.2f\n", name, us[200 + n / 2], us[200 + n / 10],
              us[200 + n * 99 / 100]);
  return 0;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "pinned";
  int khz = 100000;
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  uint32_t *ack_h = nullptr, *ack_d = nullptr;
  CK(hipHostMalloc((void**)&ack_h, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&ack_d, ack_h, 0));
  if (!std::strcmp(mode, "pinned")) {  // (a) request in pinned coherent host memory
    uint32_t *req_h = nullptr, *req_hd = nullptr;
    CK(hipHostMalloc((void**)&req_h, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&req_hd, req_h, 0));
    if (pingpong("pinned host request", req_h, req_hd, ack_h, ack_d, khz)) return 1;
  } else {  // (b) request in device memory, written by the host through the device pointer
    const bool fine = !std::strcmp(mode, "fine");
    const char* name = fine ? "device fine-grained request" : "device uncached request";
    uint32_t* d = nullptr;
    CK(hipExtMallocWithFlags((void**)&d, 1 << 20, fine ? hipDeviceMallocFinegrained : hipDeviceMallocUncached));
    hipPointerAttribute_t at;
    std::memset(&at, 0, sizeof at);
    if (hipPointerGetAttributes(&at, d) == hipSuccess)
      std::printf("%s: type %d, host pointer %p, device pointer %p\n", name, (int)at.type, at.hostPointer,
                  at.devicePointer);
    std::fflush(stdout);
    volatile uint32_t* q = d;
    q[0] = 0x5a5a5a5a;  // faults here if the host cannot reach it
    std::printf("%s: host store/load through the device pointer -> %s\n", name, q[0] == 0x5a5a5a5a ? "ok" : "wrong");
    if (pingpong(name, d, d, ack_h, ack_d, khz)) return 1;
    CK(hipFree(d));
  }
  std::printf("PROBE_OK\n");
  return 0;
}
