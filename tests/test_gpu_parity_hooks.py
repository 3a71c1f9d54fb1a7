"""Parity hooks are data, not code (-m gpu): the constants that pin parity
with the absent crates -- fastcdc 3.1.0's GEAR table, cdc-chunkers 0.1.3's
Rabin polynomial -- are installed at run time (cdc_set_gear,
cdc_set_rabin_poly) and every GPU path stays bit-exact against the oracle run
with the same constants: the device-resident pipeline, the one-launch small
kernel, the host path and the streaming write path.  Swapping in the crates'
values is therefore one call each (DESIGN.md "Oracle")."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _check(got, ref, what):
    got = np.asarray(got, dtype=np.uint64).reshape(-1, 2)
    assert got.shape == ref.shape and (got == ref).all(), what


@pytest.mark.parametrize("sizes", [(4096, 8192, 16384), (2048, 8192, 65536), (512, 2048, 16384)])
def test_second_gear_every_path(sizes):
    import torch
    import chunkfs_amd as c
    gear = oracle.splitmix64_bytes(256 * 8, 0xBEEF).view(np.uint64).copy()
    ch = c.FastChunker(c.SizeParams(*sizes))
    ch.set_gear(gear)
    data = oracle.splitmix64_bytes((64 << 20) + 4321, 99)
    ref = oracle.fastcdc(data, *sizes, gear=gear)
    assert not np.array_equal(ref, oracle.fastcdc(data, *sizes)) or ref.shape[0] < 2  # the table matters
    buf = torch.from_numpy(data).cuda()
    cap = ch.batch_max_chunks([data.size])
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda")
    first = ch.chunk_batch_device([buf.data_ptr()], [data.size], out.data_ptr(), cap)
    _check(out[:int(first[1])].cpu().numpy().view(np.uint64), ref, "device pipeline")
    for n in ((1 << 20) + 777, 3 << 20):  # one-launch small kernel (host and device input)
        r = oracle.fastcdc(data[:n], *sizes, gear=gear)
        _check(ch.chunk_array(data[:n]), r, ("host", n))
        first = ch.chunk_batch_device([buf.data_ptr()], [n], out.data_ptr(), cap)
        _check(out[:int(first[1])].cpu().numpy().view(np.uint64), r, ("device small", n))
    spans, _ = c.write_spans(ch, data[:16 << 20])
    ref_fs, _ = oracle.fs_write("fast", data[:16 << 20], *sizes, gear=gear)
    assert [int(x) for x in spans] == [int(x) for x in ref_fs]
    ch.close()


@pytest.mark.parametrize("poly", [0x2E8A2B1C4F0B35, 0xB5D3A8E2C1F3B7, 0x1D3F5C7B9])
def test_second_rabin_poly(poly):
    """A second polynomial of degree 53 (the built-in's), one of degree 55 and
    one of degree 32 (below the dword bitmap pass's range: the other path)."""
    import torch
    import chunkfs_amd as c
    sizes = c.SizeParams(2048, 4096, 8192)
    ch = c.RabinChunker(sizes)
    ch.set_poly(poly)
    data = oracle.splitmix64_bytes((32 << 20) + 123, 5)
    data[(8 << 20) + 5:(9 << 20) + 77] = 0  # a quiet run
    ref = oracle.cdc("rabin", data, 2048, 4096, 8192, rabin_poly=poly)
    assert not np.array_equal(ref, oracle.cdc("rabin", data, 2048, 4096, 8192))
    buf = torch.from_numpy(data).cuda()
    cap = ch.batch_max_chunks([data.size])
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda")
    first = ch.chunk_batch_device([buf.data_ptr()], [data.size], out.data_ptr(), cap)
    _check(out[:int(first[1])].cpu().numpy().view(np.uint64), ref, "device")
    _check(ch.chunk_array(data[:(2 << 20) + 9]), oracle.cdc("rabin", data[:(2 << 20) + 9], 2048, 4096, 8192,
                                                             rabin_poly=poly), "host")
    ch.close()


def test_rabin_poly_rules():
    import chunkfs_amd as c
    ch = c.RabinChunker(c.SizeParams(2048, 4096, 8192))
    for bad in (0, 0x1FF, 1 << 57):
        with pytest.raises(c.CdcError):
            ch.set_poly(bad)
    ch.close()
    f = c.FastChunker(c.SizeParams(4096, 8192, 16384))
    with pytest.raises(c.CdcError):
        lib = c._lib.lib()
        c._lib.check(lib.cdc_set_rabin_poly(f._h, 0x3DA3358B4DC173))
    f.close()
