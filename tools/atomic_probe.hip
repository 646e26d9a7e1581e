// Microbenchmark: throughput of agent-scope atomics on ONE address vs spread addresses.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void OneAddr(unsigned long long* c, int per_block) {
  if (threadIdx.x == 0)
    for (int i = 0; i < per_block; ++i) atomicAdd(c, 1ULL);
}
__global__ void OneAddrWave(unsigned int* c) {  // every lane adds: one wave instruction
  atomicAdd(c, 1u);
}
__global__ void Spread(unsigned long long* c, int per_block) {
  if (threadIdx.x == 0)
    for (int i = 0; i < per_block; ++i) atomicAdd(c + ((blockIdx.x * 97 + i) & 65535) * 16, 1ULL);
}
int main() {
  unsigned long long* c;
  hipMalloc(&c, 65536 * 128);
  hipMemset(c, 0, 65536 * 128);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rep = 0; rep < 2; ++rep) {
    for (int blocks : {2048, 24576}) {
      float ms;
      hipEventRecord(a);
      OneAddr<<<blocks, 64>>>(c, 1);
      hipEventRecord(b);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
      printf("one-address, %d blocks x 1 atomic: %.3f ms (%.1f ns/atomic)\n", blocks, ms, ms * 1e6 / blocks);
      hipEventRecord(a);
      OneAddr<<<blocks, 64>>>(c, 8);
      hipEventRecord(b);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
      printf("one-address, %d blocks x 8 atomics: %.3f ms (%.1f ns/atomic)\n", blocks, ms, ms * 1e6 / (blocks * 8));
      hipEventRecord(a);
      Spread<<<blocks, 64>>>(c + 8192, 8);
      hipEventRecord(b);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
      printf("spread, %d blocks x 8 atomics: %.3f ms (%.1f ns/atomic)\n", blocks, ms, ms * 1e6 / (blocks * 8));
      hipEventRecord(a);
      OneAddrWave<<<blocks, 256>>>(reinterpret_cast<unsigned int*>(c + 4096));
      hipEventRecord(b);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
      printf("one-address all lanes, %d blocks x 256: %.3f ms\n", blocks, ms);
    }
  }
  return 0;
}
