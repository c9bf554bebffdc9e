"""The per-call staging's copy kernels (srsran_amd/csrc/stage_copy.hip, behind every descriptor upload and result
read-back of the batch path and the drop-in) against numpy, over page-locked fine-grained host memory as the library
allocates it: host -> device and device -> host, source and destination offsets 0..16 (16-byte, 4-byte and
byte-aligned kernels), sizes 1 .. 70,001 bytes (tails of every length), and one multi-segment launch mixing
directions, alignments and sizes.  Bytes outside each destination range must stay untouched."""
import ctypes as C

import numpy as np
import pytest

from srsran_amd import lib

pytestmark = pytest.mark.gpu

CAP = 70_001 + 64
SIZES = [1, 2, 3, 4, 5, 7, 15, 16, 17, 31, 63, 64, 65, 255, 256, 257, 1000, 4097, 16_385, 65_535, 70_001]
OFFS = [(0, 0), (1, 0), (0, 3), (4, 4), (8, 0), (15, 7), (2, 14), (16, 16), (3, 5), (12, 4)]


def _L():
    L = lib()
    L.mi355_debug_stage_host_alloc.argtypes = [C.c_size_t]
    L.mi355_debug_stage_host_alloc.restype = C.c_void_p
    L.mi355_debug_stage_host_free.argtypes = [C.c_void_p]
    L.mi355_debug_stage_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    L.mi355_debug_stage_copy.restype = C.c_int
    return L


class Bufs:
    def __init__(self):
        from srsran_amd.tdec import DeviceBuffer
        L = _L()
        self.hp = L.mi355_debug_stage_host_alloc(CAP)
        assert self.hp
        self.host = np.ctypeslib.as_array((C.c_uint8 * CAP).from_address(self.hp))
        self.dev = DeviceBuffer(CAP, 0)

    def dev_read(self):
        return self.dev.download(np.zeros(CAP, np.uint8))

    def close(self):
        _L().mi355_debug_stage_host_free(self.hp)
        self.dev.free()


def _copy(segs):
    """segs: [(dst, src, nbytes)]; one segment -> stage_copy, several -> stage_copy_multi"""
    n = len(segs)
    dst = (C.c_void_p * n)(*[s[0] for s in segs])
    src = (C.c_void_p * n)(*[s[1] for s in segs])
    nb = (C.c_uint32 * n)(*[s[2] for s in segs])
    assert _L().mi355_debug_stage_copy(dst, src, nb, 0 if n == 1 else n) == 0


@pytest.fixture(scope="module")
def bufs():
    b = Bufs()
    yield b
    b.close()


@pytest.mark.parametrize("multi", [False, True], ids=["stage_copy", "stage_copy_multi_1seg"])
def test_h2d_offsets_and_sizes(bufs, multi):
    rng = np.random.default_rng(11)
    for od, os_ in OFFS:
        for n in SIZES:
            if max(od, os_) + n > CAP:
                continue
            src = rng.integers(0, 256, CAP, dtype=np.uint8)
            bufs.host[:] = src
            lib().mi355_memset_dev(bufs.dev.ptr, 0, CAP)
            seg = [(bufs.dev.ptr + od, bufs.hp + os_, n)]
            if multi:  # a 1-segment multi launch goes through the same kernel as several segments
                n2 = C.c_int(1)
                dst = (C.c_void_p * 1)(seg[0][0])
                srcp = (C.c_void_p * 1)(seg[0][1])
                nb = (C.c_uint32 * 1)(n)
                assert _L().mi355_debug_stage_copy(dst, srcp, nb, n2.value) == 0
            else:
                _copy(seg)
            want = np.zeros(CAP, np.uint8)
            want[od: od + n] = src[os_: os_ + n]
            assert np.array_equal(bufs.dev_read(), want), (od, os_, n)


def test_d2h_offsets_and_sizes(bufs):
    rng = np.random.default_rng(12)
    for od, os_ in OFFS:
        for n in SIZES:
            if max(od, os_) + n > CAP:
                continue
            src = rng.integers(0, 256, CAP, dtype=np.uint8)
            bufs.dev.upload(src)
            bufs.host[:] = 0
            _copy([(bufs.hp + od, bufs.dev.ptr + os_, n)])
            want = np.zeros(CAP, np.uint8)
            want[od: od + n] = src[os_: os_ + n]
            assert np.array_equal(bufs.host, want), (od, os_, n)


def test_multi_segment_launch_mixed(bufs):
    """Six segments in one launch: both directions, 16-byte / 4-byte / byte alignment, tails of several lengths."""
    from srsran_amd.tdec import DeviceBuffer
    rng = np.random.default_rng(13)
    dev2 = DeviceBuffer(CAP, 0)
    hsrc = rng.integers(0, 256, CAP, dtype=np.uint8)
    dsrc = rng.integers(0, 256, CAP, dtype=np.uint8)
    bufs.host[:] = hsrc
    dev2.upload(dsrc)
    lib().mi355_memset_dev(bufs.dev.ptr, 0, CAP)
    # h2d into bufs.dev from bufs.host, d2h into a second host region? (host is also a source): use disjoint ranges
    segs = [(bufs.dev.ptr + 0, bufs.hp + 0, 4096),          # 16-aligned
            (bufs.dev.ptr + 4100, bufs.hp + 5000, 1027),    # 4-aligned, tail 3
            (bufs.dev.ptr + 6001, bufs.hp + 7003, 2049),    # unaligned
            (bufs.dev.ptr + 9000, dev2.ptr + 123, 777),     # device -> device, unaligned
            (bufs.hp + 40_000, dev2.ptr + 20_000, 25_000),  # d2h, 16-aligned, into a host range nobody reads
            (bufs.hp + 66_001, dev2.ptr + 3, 3_999)]        # d2h, unaligned
    _copy(segs)
    wd = np.zeros(CAP, np.uint8)
    wd[0:4096] = hsrc[0:4096]
    wd[4100:5127] = hsrc[5000:6027]
    wd[6001:8050] = hsrc[7003:9052]
    wd[9000:9777] = dsrc[123:900]
    assert np.array_equal(bufs.dev_read(), wd)
    wh = hsrc.copy()
    wh[40_000:65_000] = dsrc[20_000:45_000]
    wh[66_001:70_000] = dsrc[3:4002]
    assert np.array_equal(bufs.host, wh)
    dev2.free()
