"""Test-side restatement of the device noise draw of include/ddmi.h (noise == NULL): Philox4x32-10 (Salmon,
Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3", SC'11; the Random123 round function and
key schedule) and the Box-Muller transform elementwise.hip applies to its output. Checker only."""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr, key):
    """ctr: (n, 4) uint32, key: (2,) uint32 -> (n, 4) uint32."""
    c = [ctr[:, i].astype(np.uint64) for i in range(4)]
    k0, k1 = np.uint32(key[0]), np.uint32(key[1])
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0, p1 = M0 * c[0], M1 * c[2]
            c = [(p1 >> np.uint64(32)) ^ c[1] ^ np.uint64(k0), p1 & MASK,
                 (p0 >> np.uint64(32)) ^ c[3] ^ np.uint64(k1), p0 & MASK]
            k0, k1 = np.uint32(k0 + W0), np.uint32(k1 + W1)
    return np.stack(c, 1).astype(np.uint32)


def device_normals(seed: int, first: int, n: int) -> np.ndarray:
    """Normals first .. first + n - 1 of the stream keyed by seed (first, n multiples of 4), float32."""
    g = np.arange(first // 4, (first + n) // 4, dtype=np.uint64)
    ctr = np.zeros((len(g), 4), np.uint32)
    ctr[:, 0] = (g & MASK).astype(np.uint32)
    ctr[:, 1] = (g >> np.uint64(32)).astype(np.uint32)
    x = philox4x32_10(ctr, np.array([seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF], np.uint32))
    out = np.empty((len(g), 4), np.float32)
    for h in range(2):
        u = ((x[:, 2 * h] >> np.uint32(8)).astype(np.float32) + np.float32(1)) * np.float32(2.0 ** -24)
        v = (x[:, 2 * h + 1] >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24)
        r = np.sqrt(np.float32(-2) * np.log(u))
        out[:, 2 * h] = r * np.cos(np.float32(2 * np.pi) * v)
        out[:, 2 * h + 1] = r * np.sin(np.float32(2 * np.pi) * v)
    return out.reshape(-1)
