// LDS same-address semantics on gfx950, one wave: which lane's ds_write_b8 wins when several
// lanes of one instruction store to one byte, and in which lane order ds_add_rtn_u32 to one
// address returns its old values.  Output: one line per case.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(int *out) {
    __shared__ unsigned char b[256];
    __shared__ unsigned int w[64];
    const int lane = threadIdx.x;
    b[lane] = 0xff;
    b[64 + lane] = 0xff;
    w[lane] = 0;
    __syncthreads();
    b[0] = (unsigned char)lane;                         // all 64 lanes, one byte
    if (lane & 1) b[1] = (unsigned char)lane;           // odd lanes
    if (lane >= 5 && lane < 40 && (lane % 7) == 0) b[2] = (unsigned char)lane;  // 7,14,21,28,35
    b[4 + (lane & 3)] = (unsigned char)lane;            // 16 lanes per byte, 4 bytes of one dword
    __syncthreads();
    const unsigned int old = atomicAdd(&w[0], 1u);      // ds_add_rtn_u32, same address
    const unsigned int old2 = atomicAdd(&w[1 + (lane & 1)], (unsigned)lane + 1);
    __syncthreads();
    out[lane] = (int)old;
    out[64 + lane] = (int)old2;
    if (lane < 8) out[128 + lane] = b[lane];
}

int main() {
    int *d, h[136];
    hipMalloc(&d, sizeof h);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("write_b8 winners: all=%d odd=%d sparse=%d quad={%d,%d,%d,%d}\n", h[128], h[129], h[130], h[132], h[133],
           h[134], h[135]);
    printf("ds_add_rtn old by lane:");
    for (int i = 0; i < 64; ++i) printf(" %d", h[i]);
    printf("\nds_add_rtn (two addresses, +lane+1) old by lane:");
    for (int i = 0; i < 16; ++i) printf(" %d", h[64 + i]);
    printf("\n");
    return 0;
}
