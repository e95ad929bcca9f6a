// Host check of lane::load_dw (the device board loader) against lane::load.
#include <stdint.h>
#include <string.h>
static inline uint32_t host_alignbyte(uint32_t hi, uint32_t lo, uint32_t sh)
{
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sh));
}
#define __builtin_amdgcn_alignbyte host_alignbyte
#define LS_HOST_ALIGNBYTE 1
#include "../../sudoku_solver_distributed_amd/csrc/lane_solver.h"

// boards: n*81 bytes inside a buffer padded by 8 bytes at the end;
// returns the number of boards where the two loaders disagree
extern "C" int64_t check_load_dw(const uint8_t *boards, int64_t n)
{
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) {
        lane::Board a, b;
        lane::load(a, boards + i * 81);
        const bool ok = lane::load_dw(b, boards + i * 81);
        bool valid = true;
        for (int k = 0; k < 81; ++k) valid &= boards[i * 81 + k] <= 9;
        if (ok != valid) { bad++; continue; }
        if (!valid) continue;
        if (memcmp(a.V, b.V, sizeof a.V) || memcmp(a.E, b.E, sizeof a.E) || memcmp(a.U, b.U, sizeof a.U) || a.bad != b.bad)
            bad++;
    }
    return bad;
}
