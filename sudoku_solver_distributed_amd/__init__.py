"""sudoku_solver_distributed_amd -- MI355X-native Sudoku solving.

A drop-in for the hot path of cristiano-nicolau/sudoku_solver_distributed:
the reference's backtracking solve (gen.py:6-28, node.py:62-74) and board
checks (sudoku.py:119-140, node.py:82-116), re-built as hand-written gfx950
HIP kernels behind a C ABI (include/sudoku_hip.h, libsudoku_hip.so), with the
reference's Python API surface on top:

    from sudoku_solver_distributed_amd.sudoku import Sudoku    # sudoku.py
    from sudoku_solver_distributed_amd.gen import solve_sudoku, generate_sudoku  # gen.py
    from sudoku_solver_distributed_amd.solver import BatchSolver  # (n, 81) batches
    from sudoku_solver_distributed_amd import distributed         # multi-GPU shards

Importing the package does not touch the GPU; the first solver call loads the
library and raises if it (or a GPU) is missing.
"""
__version__ = "0.1.0"

__all__ = ["__version__"]
