"""Deterministic input generator shared by the golden-vector writer and the tests (splitmix64 byte stream)."""
import numpy as np

_M64 = (1 << 64) - 1


def splitmix_u64(seed: int, n: int) -> np.ndarray:
    """n outputs of splitmix64 starting from state `seed` (vectorised: state_i = seed + (i+1)*golden)."""
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed & _M64) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def splitmix_bytes(seed: int, nbytes: int) -> bytes:
    words = splitmix_u64(seed, (nbytes + 7) // 8)
    return words.astype("<u8").tobytes()[:nbytes]
