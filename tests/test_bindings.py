"""The Python binding checks every tensor before a pointer reaches C:
wrong dtype, layout, length or device raises ValueError and nothing is launched.  CPU-only:
the structural checks run before the device check, so CPU tensors reach each rule."""
import pytest

torch = pytest.importorskip("torch")
import libapenetwork_amd as amd  # noqa: E402


def _u8(*shape):
    return torch.zeros(shape, dtype=torch.uint8)


def _i32(n):
    return torch.zeros(n, dtype=torch.int32)


def _i64(n):
    return torch.zeros(n, dtype=torch.int64)


def _raises(match, f, *a, **k):
    with pytest.raises(ValueError, match=match):
        f(*a, **k)


@pytest.mark.parametrize("fn", [amd.compress_batch, amd.decompress_batch])
def test_strided_batch_checks(fn):
    n = 4
    src, dst = _u8(n, 64), _u8(n, 96)
    _raises("dtype", fn, src.to(torch.int32), _i32(n), dst, _i32(n))
    _raises("dtype", fn, src, _i64(n), dst, _i32(n))
    _raises("dtype", fn, src, _i32(n), dst, _i32(n).float())
    _raises("contiguous", fn, _u8(n, 128)[:, ::2], _i32(n), dst, _i32(n))
    _raises("contiguous", fn, src, _i32(n), _u8(96, n).t(), _i32(n))
    _raises("2-D", fn, _u8(n * 64), _i32(n), dst, _i32(n))
    _raises("rows", fn, src, _i32(n), _u8(n + 1, 96), _i32(n))
    _raises("elements", fn, src, _i32(n - 1), dst, _i32(n))
    _raises("elements", fn, src, _i32(n), dst, _i32(n), dst_caps=_i32(n + 1))
    _raises("contiguous", fn, src, torch.zeros(2 * n, dtype=torch.int32)[::2], dst, _i32(n))
    # a row narrower than its stride: the C default cap (the stride) would run past it
    _raises("dst_caps", fn, src, _i32(n), _u8(n, 128)[:, :96], _i32(n))
    # structurally right, but host memory
    _raises("CUDA", fn, src, _i32(n), dst, _i32(n))
    _raises("CUDA", fn, src, _i32(n), _u8(n, 128)[:, :96], _i32(n), dst_caps=_i32(n))


def test_pointer_batch_checks():
    n = 3
    ok = dict(src_ptrs=_i64(n), src_sizes=_i32(n), dst_ptrs=_i64(n), caps=_i32(n), results=_i32(n))
    for f, extra in ((amd.compress_fast_ptr_batch, (1,)), (amd.compress_exact_ptr_batch, ())):
        _raises("dtype", f, _i32(n), ok["src_sizes"], ok["dst_ptrs"], ok["caps"], ok["results"], *extra)
        _raises("elements", f, ok["src_ptrs"], ok["src_sizes"], _i64(n + 1), ok["caps"], ok["results"],
                *extra)
        _raises("tensor", f, ok["src_ptrs"], ok["src_sizes"], ok["dst_ptrs"], None, ok["results"], *extra)
        _raises("CUDA", f, *ok.values(), *extra)
    _raises("dtype", amd.decompress_ptr_batch, _i64(n), _i64(n), _i64(n), _i32(n), _i32(n))
    _raises("elements", amd.decompress_partial_batch, _i64(n), _i32(n), _i64(n), _i32(n), _i32(n),
            _i32(n - 1))
    _raises("dtype", amd.decompress_dict_batch, _i64(n), _i32(n), _i64(n), _i32(n), _i32(n), _i32(n),
            _i32(n))
    _raises("dtype", amd.compress_prefix_batch, _i64(n), _i32(n), _i64(n), _i64(n), _i32(n), _i32(n))
    _raises("dtype", amd.decompress_fast_ptr_batch, _i64(n), _i32(n), _i64(n), _i32(n), _i64(n))
    _raises("dtype", amd.compress_destSize_ptr_batch, _i64(n), _i32(n), _i64(n), _i32(n), _u8(n))
    _raises("CUDA", amd.compress_destSize_scratch_ptr_batch, _i64(n), _i32(n), _i64(n), _i32(n),
            _i32(n), _u8(16))


def test_frame_checks():
    n = 4
    comp = _u8(n, 80)
    _raises("elements", amd.frame_pack, comp, _i32(n), _i64(n), _u8(1024))
    _raises("dtype", amd.frame_pack, comp, _i32(n), _i64(n + 1).int(), _u8(1024))
    _raises("nblocks", amd.decompress_frames, _u8(1024), _i64(n + 1), _u8(n, 64), _i32(n), nblocks=n + 1)
    _raises("offsets", amd.decompress_frames, _u8(1024), _i64(n), _u8(n, 64), _i32(n))
    _raises("dst_caps", amd.decompress_frames, _u8(1024), _i64(n + 1), _u8(n, 128)[:, :64], _i32(n))
    _raises("elements", amd.frame_offsets, _i32(n), _i64(n))
    _raises("row", amd.synth_blocks, _u8(n, 64), 65, 0, 1)
