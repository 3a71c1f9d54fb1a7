"""Seeded synthetic datasets of the bench harness.

The reference generates its datasets with `fio` or an unseeded `rand::rng()`
(src/bench/generator.rs:42-99); neither is reproducible offline, so the bench
and the GPU tests use these seeded generators instead:

  splitmix64_bytes  little-endian u64 words, word i = mix64(seed + (i+1) *
                    0x9E3779B97F4A7C15) -- the same bytes as the device fill
                    cdc_fill_splitmix64_device (include/chunkfs_amd.h)
  versioned_archive config 3's offline substitute for the gcc tarball
                    (scripts/download-gcc.sh needs the network): a base blob
                    and successive copies with ~1 % seeded edits each
"""
import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def splitmix64_bytes(n, seed):
    """n bytes of the splitmix64 stream of `seed` (host numpy)."""
    words = (n + 7) // 8
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (np.arange(1, words + 1, dtype=np.uint64) * _GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:n].copy()


def versioned_archive(base_bytes, versions, seed=3):
    """`versions` files: a splitmix64 base of `base_bytes` and versions-1
    successive copies, each with seeded overwrites, inserts and deletes of
    64..4095 bytes at ~1 edit per 2 KiB of edit budget (1 % of the copy)."""
    rng = np.random.default_rng(seed)
    out = [splitmix64_bytes(base_bytes, seed)]
    for _ in range(versions - 1):
        v = out[-1]
        budget = v.size // 100
        parts, pos = [], 0
        for p in np.sort(rng.choice(v.size - 8192, size=max(1, budget // 2048), replace=False)):
            if p < pos:
                continue
            parts.append(v[pos:p])
            k = int(rng.integers(64, 4096))
            op = int(rng.integers(0, 3))
            if op == 0:    # overwrite k bytes
                parts.append(rng.integers(0, 256, k, dtype=np.uint8))
                pos = p + k
            elif op == 1:  # insert k bytes
                parts.append(rng.integers(0, 256, k, dtype=np.uint8))
                pos = p
            else:          # delete k bytes
                pos = p + k
        parts.append(v[pos:])
        out.append(np.ascontiguousarray(np.concatenate(parts)))
    return out
