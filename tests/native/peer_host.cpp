// Host build of sudoku_solver_distributed_amd/csrc/peer_greedy.h (the GPU's
// reference-/solve loop) for the CPU tests: checked against the oracle's
// independent restatement (oracle_peer_solve).  Not a product path.
#include <stdint.h>
#include "../../sudoku_solver_distributed_amd/csrc/peer_greedy.h"

extern "C" void peer_host_batch(const uint8_t *in, uint8_t *out, int32_t *status, int32_t *validations, int64_t n)
{
    static peer::State s;
    for (int64_t i = 0; i < n; ++i) {
        for (int k = 0; k < 81; ++k) s.sudoku[k] = in[i * 81 + k];
        int checks = 0;
        peer::clear_node(s.node);
        status[i] = peer::run(s, checks);
        validations[i] = checks;
        for (int k = 0; k < 81; ++k) out[i * 81 + k] = s.sudoku[k];
    }
}

// one node serving the n boards in order (sdk_peer_solve_seq's loop);
// `node` is the SDK_PEER_STATE_BYTES record, in and out
extern "C" void peer_host_seq(const uint8_t *in, uint8_t *out, int32_t *status, int32_t *validations, int64_t n,
                              void *node)
{
    static peer::State s;
    s.node = *(peer::NodeState *)node;
    for (int64_t i = 0; i < n; ++i) {
        for (int k = 0; k < 81; ++k) s.sudoku[k] = in[i * 81 + k];
        int checks = 0;
        status[i] = peer::run(s, checks);
        validations[i] = checks;
        for (int k = 0; k < 81; ++k) out[i * 81 + k] = s.sudoku[k];
    }
    *(peer::NodeState *)node = s.node;
}
