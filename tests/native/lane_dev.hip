// Device dump of the lane solver's steps (debug harness): per board, the
// Board after load_dw, then after one naked pass (+ dead/placed).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include "../../sudoku_solver_distributed_amd/csrc/lane_solver.h"

__device__ void save(const lane::Board &b, uint32_t *w)
{
#pragma unroll
    for (int k = 0; k < 11; ++k) w[k] = b.V[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) w[11 + k] = b.E[k];
#pragma unroll
    for (int k = 0; k < 27; ++k) w[14 + k] = b.U[k];
    w[41] = b.bad;
}
struct Dump { uint32_t w[2][43]; uint32_t dead, placed, ok; };

__global__ void dump_kernel(const uint8_t *boards, Dump *out, int n)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    lane::Board b;
    const bool ok = lane::load_dw(b, boards + t * 81);
    Dump &d = out[t];
    d.ok = ok;
    save(b, d.w[0]);
    uint32_t dead = 0, placed = 0;
    lane::NakedPass<0>::run(b, dead, placed);
    save(b, d.w[1]);
    d.dead = dead; d.placed = placed;
}

int main()
{
    const char *bs[2] = {"342076915198235674065401238680517392923684157571923486817342569450168723236759841",
                         "084031760000562483653870021801005037570008140432197658700450812340219576125786394"};
    uint8_t h[2 * 81 + 8] = {0};
    for (int i = 0; i < 2; ++i) for (int k = 0; k < 81; ++k) h[i * 81 + k] = bs[i][k] - '0';
    uint8_t *db; Dump *dd;
    hipMalloc(&db, sizeof h); hipMalloc(&dd, 2 * sizeof(Dump));
    hipMemcpy(db, h, sizeof h, hipMemcpyHostToDevice);
    dump_kernel<<<1, 64>>>(db, dd, 2);
    Dump r[2];
    hipMemcpy(r, dd, sizeof r, hipMemcpyDeviceToHost);
    for (int i = 0; i < 2; ++i) {
        lane::Board a; lane::load(a, h + i * 81);
        const uint32_t *s = (const uint32_t *)&a;
        printf("board %d ok=%u dead=%u placed=%u\n", i, r[i].ok, r[i].dead, r[i].placed);
        for (int k = 0; k < 42; ++k)
            if (s[k] != r[i].w[0][k]) printf("  load word %d host %08x dev %08x\n", k, s[k], r[i].w[0][k]);
        uint32_t dead = 0, placed = 0;
        lane::NakedPass<0>::run(a, dead, placed);
        printf("  host dead=%u placed=%u\n", dead, placed);
        for (int k = 0; k < 42; ++k)
            if (s[k] != r[i].w[1][k]) printf("  naked word %d host %08x dev %08x\n", k, s[k], r[i].w[1][k]);
    }
    return 0;
}
