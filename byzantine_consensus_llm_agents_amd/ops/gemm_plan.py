"""Which GEMM runs where: the hand MFMA kernel (csrc/kernels/gemm.hip) or hipBLASLt.

Decode projections are skinny (M = live rows of a decode bucket, 1..768) and
the hand kernel's tile shapes, fused epilogues and XCD-aware order are built
for them; prefill chunks (M = 16384) stay on hipBLASLt's tuned kernels.  The
choice per (M, N, K, epilogue) comes from a table measured on the GPU
(``tools/tune_hand_gemm.py`` -> ``engine/tuned/hand_gemm.json``: for every
decode bucket and projection shape, every tile configuration and the library
are timed and the fastest is kept).  Shapes the table does not cover use a
simple rule (hand kernel up to ``max_m`` rows).

``BCG_HAND_GEMM``: ``0`` = library only, ``1`` (default) = table / rule,
``force`` = hand kernel wherever the shape is supported (tests; ``BCG_HAND_GEMM_SPLIT``
= the split-K to force with it).

"""

import ctypes
import json
import os
from typing import Dict, Optional, Tuple

TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "engine", "tuned",
                     "hand_gemm.json")
TILES = ((128, 128), (64, 128), (128, 64), (256, 128), (64, 256), (64, 64), (32, 128),  # csrc/kernels/gemm.hip CFGS
         (256, 128), (128, 256), (128, 128), (256, 256), (256, 256))
PP_CFG = 10  # csrc/kernels/gemm_pp.hip: 256 x 256 ping-pong tile, N only a multiple of 16
W4_CFG = 11  # csrc/kernels/gemm_w4.hip: 256 x 256, four 128 x 128 waves (one per SIMD), LDS-DMA fed
BIG_CFGS = (PP_CFG, W4_CFG)  # 256 x 256 tiles (the register-staged form lost its A/B: csrc/experimental/gemm_rs.hip)
N_CFGS = len(TILES)
SPLITS = (1, 2, 3, 4, 6, 8)
STREAM_K = 0  # split_k value of the W4 kernel's stream-K launch (one workgroup per CU over tiles x K-tiles)


class GemmPlan:
    def __init__(self, lib=None, table: Optional[str] = TABLE, max_m: int = 1024):
        self.mode = os.environ.get("BCG_HAND_GEMM", "1")
        self.force_split = int(os.environ.get("BCG_HAND_GEMM_SPLIT", "1"))  # split-K in "force" mode (tests)
        self.max_m = max_m
        self.timings: Dict[Tuple[int, int, int, int], Dict[str, float]] = {}
        self.tiles = {}
        for cfg in range(N_CFGS):
            self.tiles[cfg] = TILES[cfg]
            if lib is not None:  # the library is the source of truth
                bm, bn = ctypes.c_int(), ctypes.c_int()
                if lib.bcg_gemm_tile(cfg, ctypes.byref(bm), ctypes.byref(bn)) == 0:
                    self.tiles[cfg] = (bm.value, bn.value)
        self.table: Dict[Tuple[int, int, int, int], Tuple[int, int]] = {}
        if table and os.path.exists(table):
            with open(table) as fh:
                data = json.load(fh)
            for key, choice in data.get("choice", {}).items():
                m, n, k, e = map(int, key.split(","))
                self.table[(m, n, k, e)] = tuple(choice) if isinstance(choice, list) else (int(choice), 1)
            for key, times in data.get("timings_us", {}).items():
                self.timings[tuple(map(int, key.split(",")))] = times

    def supported(self, cfg: int, M: int, N: int, K: int, epi: int, split_k: int = 1) -> bool:
        if split_k == STREAM_K:  # W4 only: an arrival counter per tile, 32-bit unit arithmetic
            tiles = -(-M // 256) * -(-N // 256)
            if cfg != W4_CFG or tiles > 65024 or tiles * (K // 64) * 256 >= 1 << 31:
                return False
            split_k = 1
        if cfg not in self.tiles or M <= 0 or K % 64 or K <= 0 or split_k < 1 or K // 64 < split_k:
            return False
        if cfg == W4_CFG and split_k > 1 and -(-M // 256) * -(-N // 256) > 65024:
            return False  # split-K arrival counters below the reduce-scatter scheme's slots
        bn = self.tiles[cfg][1]
        if cfg in BIG_CFGS:  # 32-bit buffer offsets: operands below 4 GiB (W4: 2 GiB), output below 2 GiB
            lim = 1 << (31 if cfg == W4_CFG else 32)
            ldc = N // 2 if epi == 1 else N
            return (N % 16 == 0 and 2 * (M + 256) * K < lim and 2 * (N + 256) * K < lim
                    and 2 * (M + 256) * ldc < 1 << 31
                    and (epi != 1 or (N % 2 == 0 and (N // 2) % 128 == 0)))
        if N % bn:
            return False
        if epi == 1 and (N % 2 or (N // 2) % (bn // 2)):
            return False
        return True

    def default_cfg(self, M: int) -> int:
        return 1 if M <= 64 else 0

    def _lookup(self, M: int, N: int, K: int, epi: int) -> Optional[Tuple[int, int]]:
        """Table choice at M, else at the nearest measured M above (same projection shape)."""
        choice = self.table.get((M, N, K, epi))
        if choice is None and self.table:
            above = [m for (m, n, k, e) in self.table if (n, k, e) == (N, K, epi) and m >= M]
            if above:
                choice = self.table[(min(above), N, K, epi)]
        return choice

    def choose(self, M: int, N: int, K: int, epi: int) -> Optional[Tuple[int, int]]:
        """(tile configuration, split-K) of the hand kernel, or None for the library path."""
        if self.mode == "0":
            return None
        if self.mode == "force":
            for cfg in (self.default_cfg(M),) + tuple(range(N_CFGS)):
                for split in ((self.force_split, 1) if self.force_split > 1 else (1,)):
                    if self.supported(cfg, M, N, K, epi, split):
                        return (cfg, split)
            return None
        choice = self._lookup(M, N, K, epi)
        if choice is None and epi in (0, 2):
            # the store and residual epilogues run the same tile loop: a shape measured with one
            # (e.g. the TP row-parallel o / down projections, tuned with the residual epilogue
            # but called with the store epilogue before the fused all-reduce) takes that choice
            choice = self._lookup(M, N, K, 2 - epi)
        if choice is not None:
            return choice if choice[0] >= 0 and self.supported(choice[0], M, N, K, epi, choice[1]) else None
        if M > self.max_m or self.table:  # a measured table exists: unlisted shapes stay on the library
            return None
        cfg = self.default_cfg(M)
        return (cfg, 1) if self.supported(cfg, M, N, K, epi) else None


FP8_TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "engine", "tuned",
                         "hand_gemm_fp8.json")
FP8_RULE_MAX_M = 128  # unmeasured shapes: the hand fp8 kernel up to this M (it won every measured M <= 128)


class Fp8Plan:
    """Which fp8 projection GEMM runs: the hand block-scaled MFMA kernel (gemm.hip, F8) or
    hipBLASLt's ``torch._scaled_mm``.  Measured shapes (``engine/tuned/hand_gemm_fp8.json``,
    ``tools/bench_fp8_gemm.py``): the choice at the nearest measured M >= M, the library
    beyond the largest measured M; unmeasured shapes: the hand kernel up to FP8_RULE_MAX_M."""

    def __init__(self, tiles: Dict[int, Tuple[int, int]], table: Optional[str] = FP8_TABLE):
        self.tiles = tiles
        self.table: Dict[Tuple[int, int, int], Tuple[int, int]] = {}
        if table and os.path.exists(table):
            with open(table) as fh:
                for key, ch in json.load(fh).get("choice", {}).items():
                    self.table[tuple(map(int, key.split(",")))] = tuple(ch)

    def choose(self, M: int, N: int, K: int) -> Optional[Tuple[int, int]]:
        if os.environ.get("BCG_HAND_GEMM", "1") == "0" or K % 128 or M <= 0:
            return None
        above = [m for (m, n, k) in self.table if (n, k) == (N, K) and m >= M]
        if above:
            cfg, split = self.table[(min(above), N, K)]
        elif any((n, k) == (N, K) for (_, n, k) in self.table) or M > FP8_RULE_MAX_M:
            return None
        else:
            cfg, split = (6 if M <= 32 else 1 if M <= 64 else 0), 1
        if cfg < 0 or cfg not in self.tiles or K // 128 < split:
            return None
        if cfg == PP_CFG:  # 256 x 256 ping-pong fp8 kernel (prefill M): N % 16, 32-bit buffer offsets
            ok = N % 16 == 0 and M * K < 1 << 32 and N * K < 1 << 32 and 2 * (M + 256) * N < 1 << 31
        elif cfg == W4_CFG:  # four-wave 256 x 256 fp8 kernel: N % 16, offsets below 2 GiB
            ok = (N % 16 == 0 and (M + 256) * K < 1 << 31 and (N + 256) * K < 1 << 31
                  and 2 * (M + 256) * N < 1 << 31)
        else:
            ok = N % self.tiles[cfg][1] == 0
        return (cfg, split) if ok else None
