"""libapenetwork_amd -- MI355X-native LZ4 block codec behind libapenetwork's ape_lz4.h.

The product is the C shared library ``libape_lz4_amd.so`` built next to this file
(``make -C libapenetwork_amd/csrc``): it exports the reference's ape_lz4.h ABI
(src/ape_lz4.h:59-467) -- one-shot calls on its host codec by default,
on HIP kernels when ``set_oneshot_host_below`` selects them -- and the batched device
API of include/ape_lz4_gpu.h, whose codec is HIP kernels only.  This module is a thin ctypes
mirror of that ABI for tests and the benchmark -- same function names, same
argument meaning, same return conventions.  There is no Python or CPU fallback:
importing works anywhere, but every call that needs the library raises if it is
missing, and GPU entry points return the library's error codes without a GPU.
"""
import ctypes as _C
import os as _os

__all__ = [
    "lib", "versionNumber", "compressBound", "compress_default", "compress_fast",
    "decompress_safe", "decompress_safe_partial", "compress_batch", "decompress_batch",
    "decompress_partial_batch", "synth_blocks", "gpu_init", "gpu_last_error", "GpuError",
    "MAX_BLOCK", "ERANGE", "frame_offsets", "frame_pack", "decompress_frames",
    "compress_prefix_batch", "decompress_dict_batch", "compress_fast_ptr_batch", "compress_exact_ptr_batch",
    "decompress_fast_ptr_batch", "compress_destSize_ptr_batch", "RxBuf",
    "compress_destSize_scratch_ptr_batch", "destSize_scratch_size",
    "socket_send_blocks", "socket_recv_blocks", "socket_stats", "set_oneshot_host_below",
    "Chain",
    "oneshot_on_gpu",
    "ONESHOT_HOST_ALL",
]

_HERE = _os.path.dirname(_os.path.abspath(__file__))
# APE_LZ4_LIB selects the diagnostic phase-timer build (tools/phase_stats.py) only.
LIB_PATH = _os.environ.get("APE_LZ4_LIB") or _os.path.join(_HERE, "libape_lz4_amd.so")
MAX_BLOCK = 65536
ERANGE = -2147483648
ONESHOT_HOST_ALL = 0x7FFFFFFF   # default one-shot threshold: every one-shot call on the host

_lib = None


class GpuError(RuntimeError):
    pass


def lib():
    """Load libape_lz4_amd.so (raises OSError with the build command if absent)."""
    global _lib
    if _lib is None:
        if not _os.path.exists(LIB_PATH):
            raise OSError("libape_lz4_amd.so not built: run `make -C %s/csrc` "
                          "(or __graft_entry__.build())" % _HERE)
        L = _C.CDLL(LIB_PATH)
        i, p, cp = _C.c_int, _C.c_void_p, _C.c_char_p
        sz, ll = _C.c_size_t, _C.c_longlong
        sig = {
            "APE_LZ4_versionNumber": (i, []),
            "APE_LZ4_compressBound": (i, [i]),
            "APE_LZ4_compress_default": (i, [p, p, i, i]),
            "APE_LZ4_compress_fast": (i, [p, p, i, i, i]),
            "APE_LZ4_decompress_safe": (i, [p, p, i, i]),
            "APE_LZ4_decompress_safe_partial": (i, [p, p, i, i, i]),
            "APE_LZ4_gpu_init": (i, []),
            "APE_LZ4_gpu_device_count": (i, []),
            "APE_LZ4_gpu_last_error": (cp, []),
            "APE_LZ4_gpu_set_oneshot_host_below": (i, [i]),
            "APE_LZ4_compress_batch_dev": (i, [p, p, p, p, p, i, p]),
            "APE_LZ4_compress_fast_batch_dev": (i, [p, p, p, p, p, i, i, p]),
            "APE_LZ4_compress_exact_batch_dev": (i, [p, p, p, p, p, i, i, p]),
            "APE_LZ4_compress_destSize_batch_dev": (i, [p, p, p, p, p, i, p]),
            "APE_LZ4_compress_destSize_scratch_size": (sz, [i]),
            "APE_LZ4_compress_destSize_batch_scratch_dev": (i, [p, p, p, p, p, i, p, sz, p]),
            "APE_LZ4_decompress_fast_batch_dev": (i, [p, p, p, p, p, i, p]),
            "APE_LZ4_decompress_safe_batch_dev": (i, [p, p, p, p, p, i, p]),
            "APE_LZ4_decompress_safe_partial_batch_dev": (i, [p, p, p, p, p, p, i, p]),
            "APE_LZ4_compress_batch_strided_dev": (i, [p, sz, p, p, sz, p, p, i, p]),
            "APE_LZ4_decompress_safe_batch_strided_dev": (i, [p, sz, p, p, sz, p, p, i, p]),
            "APE_LZ4_synth_blocks_dev": (i, [p, sz, i, ll, i, i, p]),
            "APE_LZ4_frame_scratch_size": (sz, [i]),
            "APE_LZ4_frame_offsets_dev": (i, [p, p, p, i, p]),
            "APE_LZ4_frame_pack_strided_dev": (i, [p, sz, p, p, p, i, p]),
            "APE_LZ4_decompress_safe_frames_dev": (i, [p, p, p, sz, p, p, i, p]),
            "APE_LZ4_compress_withPrefix_batch_dev": (i, [p, p, p, p, p, p, i, p]),
            "APE_LZ4_decompress_safe_usingDict_batch_dev": (i, [p, p, p, p, p, p, p, i, p]),
            "APE_LZ4_rxbuf_new": (p, [sz]),
            "APE_LZ4_rxbuf_prepare": (i, [p, sz]),
            "APE_LZ4_rxbuf_append": (i, [p, p, sz]),
            "APE_LZ4_rxbuf_frames": (i, [p, p, i, i]),
            "APE_LZ4_rxbuf_consume": (None, [p, sz]),
            "APE_LZ4_rxbuf_data": (p, [p]),
            "APE_LZ4_rxbuf_used": (sz, [p]),
            "APE_LZ4_rxbuf_room": (sz, [p]),
            "APE_LZ4_rxbuf_pinned": (i, [p]),
            "APE_LZ4_rxbuf_free": (None, [p]),
            "APE_LZ4_socket_send_blocks": (ll, [i, p, sz, i, i, i]),
            "APE_LZ4_socket_recv_blocks": (ll, [i, p, sz, i, i, i, p]),
            "APE_LZ4_socket_stats": (i, [p, i]),
            "APE_LZ4_chain_new": (p, [i, i]),
            "APE_LZ4_chain_free": (None, [p]),
            "APE_LZ4_chain_send": (ll, [p, p, p, sz, i]),
            "APE_LZ4_chain_recv": (ll, [p, p, p, sz, i, p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _lib = L
    return _lib


def versionNumber():
    return lib().APE_LZ4_versionNumber()


def compressBound(n):
    return lib().APE_LZ4_compressBound(n)


def gpu_init():
    return lib().APE_LZ4_gpu_init()


def gpu_last_error():
    s = lib().APE_LZ4_gpu_last_error()
    return s.decode() if s else ""


def set_oneshot_host_below(nbytes):
    """APE_LZ4_gpu_set_oneshot_host_below: one-shot calls on blocks smaller than nbytes run
    the host codec, larger ones the GPU (0 = all on the GPU).  Returns the previous value."""
    return lib().APE_LZ4_gpu_set_oneshot_host_below(nbytes)


class oneshot_on_gpu:
    """Context manager: route every one-shot call to the GPU path inside the block."""

    def __enter__(self):
        self._prev = set_oneshot_host_below(0)
        return self

    def __exit__(self, *exc):
        set_oneshot_host_below(self._prev)
        return False


def _buf(b, pad=16):
    return _C.create_string_buffer(bytes(b) + b"\0" * pad, len(b) + pad)


# ---- one-shot ape_lz4.h calls (host buffers; host codec or GPU, see above) ----
def compress_default(src, max_dst=None):
    """APE_LZ4_compress_default: returns (ret, compressed_bytes)."""
    cap = compressBound(len(src)) if max_dst is None else max_dst
    out = _C.create_string_buffer(max(cap, 1))
    r = lib().APE_LZ4_compress_default(_buf(src), out, len(src), cap)
    return r, out.raw[:max(r, 0)]


def compress_fast(src, max_dst=None, acceleration=1):
    cap = compressBound(len(src)) if max_dst is None else max_dst
    out = _C.create_string_buffer(max(cap, 1))
    r = lib().APE_LZ4_compress_fast(_buf(src), out, len(src), cap, acceleration)
    return r, out.raw[:max(r, 0)]


def decompress_safe(comp, max_out):
    """APE_LZ4_decompress_safe: returns (ret, dst[0:ret])."""
    out = _C.create_string_buffer(max(max_out, 1))
    r = lib().APE_LZ4_decompress_safe(_buf(comp), out, len(comp), max_out)
    return r, out.raw[:max(r, 0)]


def decompress_safe_partial(comp, target, max_out):
    out = _C.create_string_buffer(max(max_out, 1))
    r = lib().APE_LZ4_decompress_safe_partial(_buf(comp), out, len(comp), target, max_out)
    return r, out.raw[:max(r, 0)]


# ---- batched device API on torch tensors (device-resident) ----
def _ptr(t):
    return None if t is None else _C.c_void_p(t.data_ptr())


def _stream(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return _C.c_void_p(stream.cuda_stream)


def _check(rc, what):
    if rc != 0:
        raise GpuError("%s failed (%d): %s" % (what, rc, gpu_last_error()))


# ---- argument checks: every pointer handed to C comes from a tensor of the dtype, device and
# layout the C signature assumes; ValueError before any call ----
def _arr(t, what, dtype, n=None, optional=False, cuda=True):
    """A contiguous 1-D CUDA tensor of `dtype` (and length n when given)."""
    import torch
    if t is None and optional:
        return
    if not isinstance(t, torch.Tensor):
        raise ValueError("%s: need a torch tensor" % what)
    if t.dtype != dtype:
        raise ValueError("%s: dtype %s, need %s" % (what, t.dtype, dtype))
    if t.dim() != 1 or not t.is_contiguous():
        raise ValueError("%s: need a contiguous 1-D tensor" % what)
    if n is not None and t.shape[0] != n:
        raise ValueError("%s: %d elements, need %d" % (what, t.shape[0], n))
    if cuda:
        _on_cuda(what, t)


def _rows(t, what, n=None, cuda=True):
    """A 2-D uint8 CUDA tensor whose rows are contiguous (row i at data_ptr + i * stride(0),
    shape[1] bytes each, rows not overlapping)."""
    import torch
    if not isinstance(t, torch.Tensor):
        raise ValueError("%s: need a torch tensor" % what)
    if t.dtype != torch.uint8:
        raise ValueError("%s: dtype %s, need torch.uint8" % (what, t.dtype))
    if t.dim() != 2:
        raise ValueError("%s: need a 2-D tensor [blocks, bytes]" % what)
    if (t.shape[1] > 1 and t.stride(1) != 1) or (t.shape[0] > 1 and t.stride(0) < t.shape[1]):
        raise ValueError("%s: rows must be contiguous and not overlap" % what)
    if n is not None and t.shape[0] != n:
        raise ValueError("%s: %d rows, need %d" % (what, t.shape[0], n))
    if cuda:
        _on_cuda(what, t)


def _on_cuda(what, *ts):
    for t in ts:
        if t is not None and t.device.type != "cuda":
            raise ValueError("%s: need CUDA tensors" % what)


def _strided_args(src, sizes, dst, results, caps, what):
    """compress_batch / decompress_batch: the C side reads block i at src + i*stride(0) and
    writes dst + i*stride(0) with capacity caps[i] or, without caps, stride(0) -- so a row
    narrower than its stride needs explicit caps."""
    import torch
    _rows(src, what + " src", cuda=False)
    n = src.shape[0]
    _rows(dst, what + " dst", n, cuda=False)
    _arr(sizes, what + " sizes", torch.int32, n, cuda=False)
    _arr(results, what + " results", torch.int32, n, cuda=False)
    _arr(caps, what + " dst_caps", torch.int32, n, optional=True, cuda=False)
    if caps is None and n > 0 and dst.shape[1] != dst.stride(0):
        raise ValueError("%s: dst rows narrower than their stride need dst_caps" % what)
    _on_cuda(what, src, dst, sizes, results, caps)
    return n


def _ptr_args(what, n, **arrs):
    """Pointer-array calls: name -> (tensor, dtype) of N elements each (int64 pointers, int32
    sizes); a None tensor is allowed where dtype is given as (dtype, True)."""
    for name, (t, spec) in arrs.items():
        dtype, opt = spec if isinstance(spec, tuple) else (spec, False)
        _arr(t, "%s %s" % (what, name), dtype, n, optional=opt, cuda=False)
    _on_cuda(what, *(t for t, _ in arrs.values()))


def _i64():
    import torch
    return torch.int64


def _i32():
    import torch
    return torch.int32


def compress_batch(src, src_sizes, dst, results, dst_caps=None, stream=None):
    """N x APE_LZ4_compress_default on device.

    src: uint8 [N, S] CUDA tensor (block i = row i, first src_sizes[i] bytes);
    dst: uint8 [N, D] CUDA tensor; results: int32 [N] (compressed size or 0).
    """
    n = _strided_args(src, src_sizes, dst, results, dst_caps, "compress_batch")
    _check(lib().APE_LZ4_compress_batch_strided_dev(
        _ptr(src), src.stride(0), _ptr(src_sizes), _ptr(dst), dst.stride(0), _ptr(dst_caps),
        _ptr(results), n, _stream(stream)), "APE_LZ4_compress_batch_strided_dev")


def decompress_batch(comp, comp_sizes, dst, results, dst_caps=None, stream=None):
    """N x APE_LZ4_decompress_safe on device (caps default to dst row stride)."""
    n = _strided_args(comp, comp_sizes, dst, results, dst_caps, "decompress_batch")
    _check(lib().APE_LZ4_decompress_safe_batch_strided_dev(
        _ptr(comp), comp.stride(0), _ptr(comp_sizes), _ptr(dst), dst.stride(0), _ptr(dst_caps),
        _ptr(results), n, _stream(stream)), "APE_LZ4_decompress_safe_batch_strided_dev")


def decompress_partial_batch(src_ptrs, comp_sizes, dst_ptrs, targets, caps, results,
                             stream=None):
    """N x APE_LZ4_decompress_safe_partial, pointer-array form (int64 tensors of pointers)."""
    n = comp_sizes.shape[0]
    _ptr_args("decompress_partial_batch", n, src_ptrs=(src_ptrs, _i64()), comp_sizes=(comp_sizes, _i32()),
              dst_ptrs=(dst_ptrs, _i64()), targets=(targets, _i32()), caps=(caps, _i32()),
              results=(results, _i32()))
    _check(lib().APE_LZ4_decompress_safe_partial_batch_dev(
        _ptr(src_ptrs), _ptr(comp_sizes), _ptr(dst_ptrs), _ptr(targets), _ptr(caps),
        _ptr(results), n, _stream(stream)), "APE_LZ4_decompress_safe_partial_batch_dev")


def compress_fast_ptr_batch(src_ptrs, src_sizes, dst_ptrs, caps, results, acceleration,
                            stream=None):
    """N x APE_LZ4_compress_fast, pointer-array form (int64 tensors of pointers)."""
    n = src_sizes.shape[0]
    _ptr_args("compress_fast_ptr_batch", n, src_ptrs=(src_ptrs, _i64()), src_sizes=(src_sizes, _i32()),
              dst_ptrs=(dst_ptrs, _i64()), caps=(caps, _i32()), results=(results, _i32()))
    _check(lib().APE_LZ4_compress_fast_batch_dev(
        _ptr(src_ptrs), _ptr(src_sizes), _ptr(dst_ptrs), _ptr(caps), _ptr(results), n,
        acceleration, _stream(stream)), "APE_LZ4_compress_fast_batch_dev")


def compress_exact_ptr_batch(src_ptrs, src_sizes, dst_ptrs, caps, results, acceleration=1,
                             stream=None):
    """Greedy-exact mode: N x APE_LZ4_compress_fast byte for byte (the reference's own
    sequential parse, one wave per block; slow, for debugging)."""
    n = src_sizes.shape[0]
    _ptr_args("compress_exact_ptr_batch", n, src_ptrs=(src_ptrs, _i64()), src_sizes=(src_sizes, _i32()),
              dst_ptrs=(dst_ptrs, _i64()), caps=(caps, _i32()), results=(results, _i32()))
    _check(lib().APE_LZ4_compress_exact_batch_dev(
        _ptr(src_ptrs), _ptr(src_sizes), _ptr(dst_ptrs), _ptr(caps), _ptr(results), n,
        acceleration, _stream(stream)), "APE_LZ4_compress_exact_batch_dev")


def compress_destSize_ptr_batch(src_ptrs, src_sizes, dst_ptrs, targets, results, stream=None):
    """N x APE_LZ4_compress_destSize, pointer-array form: src_sizes (int32) is in/out --
    input sizes on entry, consumed input bytes on return; results = bytes written."""
    n = src_sizes.shape[0]
    _ptr_args("compress_destSize_ptr_batch", n, src_ptrs=(src_ptrs, _i64()),
              src_sizes=(src_sizes, _i32()), dst_ptrs=(dst_ptrs, _i64()), targets=(targets, _i32()),
              results=(results, _i32()))
    _check(lib().APE_LZ4_compress_destSize_batch_dev(
        _ptr(src_ptrs), _ptr(src_sizes), _ptr(dst_ptrs), _ptr(targets), _ptr(results), n,
        _stream(stream)), "APE_LZ4_compress_destSize_batch_dev")


def compress_destSize_scratch_ptr_batch(src_ptrs, src_sizes, dst_ptrs, targets, results,
                                        scratch, stream=None):
    """compress_destSize_ptr_batch with caller-owned scratch (uint8 CUDA tensor of at least
    destSize_scratch_size(1) bytes): allocates nothing, so it can be graph-captured."""
    n = src_sizes.shape[0]
    _ptr_args("compress_destSize_scratch_ptr_batch", n, src_ptrs=(src_ptrs, _i64()),
              src_sizes=(src_sizes, _i32()), dst_ptrs=(dst_ptrs, _i64()), targets=(targets, _i32()),
              results=(results, _i32()))
    import torch
    _arr(scratch, "compress_destSize_scratch_ptr_batch scratch", torch.uint8)
    _check(lib().APE_LZ4_compress_destSize_batch_scratch_dev(
        _ptr(src_ptrs), _ptr(src_sizes), _ptr(dst_ptrs), _ptr(targets), _ptr(results), n,
        _ptr(scratch), scratch.numel(), _stream(stream)),
        "APE_LZ4_compress_destSize_batch_scratch_dev")


def destSize_scratch_size(nblocks):
    return lib().APE_LZ4_compress_destSize_scratch_size(nblocks)


def decompress_fast_ptr_batch(src_ptrs, src_bounds, dst_ptrs, original_sizes, results,
                              stream=None):
    """N x APE_LZ4_decompress_fast, pointer-array form: results = input bytes consumed."""
    n = original_sizes.shape[0]
    _ptr_args("decompress_fast_ptr_batch", n, src_ptrs=(src_ptrs, _i64()),
              src_bounds=(src_bounds, _i32()), dst_ptrs=(dst_ptrs, _i64()),
              original_sizes=(original_sizes, _i32()), results=(results, _i32()))
    _check(lib().APE_LZ4_decompress_fast_batch_dev(
        _ptr(src_ptrs), _ptr(src_bounds), _ptr(dst_ptrs), _ptr(original_sizes), _ptr(results),
        n, _stream(stream)), "APE_LZ4_decompress_fast_batch_dev")


def decompress_ptr_batch(src_ptrs, comp_sizes, dst_ptrs, caps, results, stream=None):
    """N x APE_LZ4_decompress_safe, pointer-array form."""
    n = comp_sizes.shape[0]
    _ptr_args("decompress_ptr_batch", n, src_ptrs=(src_ptrs, _i64()), comp_sizes=(comp_sizes, _i32()),
              dst_ptrs=(dst_ptrs, _i64()), caps=(caps, _i32()), results=(results, _i32()))
    _check(lib().APE_LZ4_decompress_safe_batch_dev(
        _ptr(src_ptrs), _ptr(comp_sizes), _ptr(dst_ptrs), _ptr(caps), _ptr(results), n,
        _stream(stream)), "APE_LZ4_decompress_safe_batch_dev")


def compress_prefix_batch(src_ptrs, src_sizes, prefix_sizes, dst_ptrs, caps, results,
                          stream=None):
    """N chained-stream chunks (compress_fast_continue on a stream whose history is the
    prefix_sizes[i] bytes just before src_ptrs[i]); pointer-array form (int64 tensors)."""
    n = src_sizes.shape[0]
    _ptr_args("compress_prefix_batch", n, src_ptrs=(src_ptrs, _i64()), src_sizes=(src_sizes, _i32()),
              prefix_sizes=(prefix_sizes, _i32()), dst_ptrs=(dst_ptrs, _i64()),
              caps=(caps, _i32()), results=(results, _i32()))
    _check(lib().APE_LZ4_compress_withPrefix_batch_dev(
        _ptr(src_ptrs), _ptr(src_sizes), _ptr(prefix_sizes), _ptr(dst_ptrs), _ptr(caps),
        _ptr(results), n, _stream(stream)), "APE_LZ4_compress_withPrefix_batch_dev")


def decompress_dict_batch(src_ptrs, comp_sizes, dst_ptrs, caps, dict_ptrs, dict_sizes, results,
                          stream=None):
    """N x APE_LZ4_decompress_safe_usingDict, pointer-array form (int64 tensors)."""
    n = comp_sizes.shape[0]
    _ptr_args("decompress_dict_batch", n, src_ptrs=(src_ptrs, _i64()), comp_sizes=(comp_sizes, _i32()),
              dst_ptrs=(dst_ptrs, _i64()), caps=(caps, _i32()), dict_ptrs=(dict_ptrs, _i64()),
              dict_sizes=(dict_sizes, _i32()), results=(results, _i32()))
    _check(lib().APE_LZ4_decompress_safe_usingDict_batch_dev(
        _ptr(src_ptrs), _ptr(comp_sizes), _ptr(dst_ptrs), _ptr(caps), _ptr(dict_ptrs),
        _ptr(dict_sizes), _ptr(results), n, _stream(stream)),
        "APE_LZ4_decompress_safe_usingDict_batch_dev")


def synth_blocks(dst, block_size, first_block, kind, stream=None):
    """Fill rows of uint8 [N, S] CUDA tensor with SURVEY App. C blocks (kind 0 rand, 1 comp)."""
    _rows(dst, "synth_blocks dst", cuda=False)
    if not 0 <= block_size <= dst.shape[1]:
        raise ValueError("synth_blocks: block_size must fit a row")
    _on_cuda("synth_blocks", dst)
    _check(lib().APE_LZ4_synth_blocks_dev(_ptr(dst), dst.stride(0), block_size, first_block,
                                          dst.shape[0], kind, _stream(stream)),
           "APE_LZ4_synth_blocks_dev")


# ---- framed stream of independent blocks (include/ape_lz4_gpu.h, socket path) ----
def frame_offsets(comp_sizes, offsets, scratch=None, stream=None):
    """offsets (int64 [N+1] CUDA) <- exclusive scan of 4 + comp_sizes[i]; returns scratch."""
    import torch
    _arr(comp_sizes, "frame_offsets comp_sizes", torch.int32, cuda=False)
    n = comp_sizes.shape[0]
    _arr(offsets, "frame_offsets offsets", torch.int64, n + 1, cuda=False)
    if scratch is not None:
        _arr(scratch, "frame_offsets scratch", torch.uint8, cuda=False)
        if scratch.numel() < lib().APE_LZ4_frame_scratch_size(n):
            raise ValueError("frame_offsets: scratch smaller than APE_LZ4_frame_scratch_size")
    _on_cuda("frame_offsets", comp_sizes, offsets, scratch)
    if scratch is None:
        nbytes = lib().APE_LZ4_frame_scratch_size(n)
        scratch = torch.empty(max(nbytes, 8), dtype=torch.uint8, device=comp_sizes.device)
    _check(lib().APE_LZ4_frame_offsets_dev(_ptr(comp_sizes), _ptr(offsets), _ptr(scratch), n,
                                           _stream(stream)), "APE_LZ4_frame_offsets_dev")
    return scratch


def frame_pack(comp, comp_sizes, offsets, frames, stream=None):
    """Framed stream [le32 c][c bytes]... of the compressed rows of comp (uint8 [N, D])."""
    import torch
    _rows(comp, "frame_pack comp", cuda=False)
    n = comp.shape[0]
    _arr(comp_sizes, "frame_pack comp_sizes", torch.int32, n, cuda=False)
    _arr(offsets, "frame_pack offsets", torch.int64, n + 1, cuda=False)
    _arr(frames, "frame_pack frames", torch.uint8, cuda=False)
    _on_cuda("frame_pack", comp, comp_sizes, offsets, frames)
    _check(lib().APE_LZ4_frame_pack_strided_dev(_ptr(comp), comp.stride(0), _ptr(comp_sizes),
                                                _ptr(offsets), _ptr(frames), n, _stream(stream)),
           "APE_LZ4_frame_pack_strided_dev")


def decompress_frames(frames, offsets, dst, results, dst_caps=None, nblocks=None, stream=None):
    """N x APE_LZ4_decompress_safe of the blocks of a framed stream into rows of dst."""
    import torch
    _rows(dst, "decompress_frames dst", cuda=False)
    n = dst.shape[0] if nblocks is None else nblocks
    if not 0 <= n <= dst.shape[0]:
        raise ValueError("decompress_frames: nblocks must be within dst's rows")
    _arr(frames, "decompress_frames frames", torch.uint8, cuda=False)
    _arr(offsets, "decompress_frames offsets", torch.int64, cuda=False)
    if offsets.shape[0] < n + 1:
        raise ValueError("decompress_frames: offsets need nblocks + 1 entries")
    _arr(results, "decompress_frames results", torch.int32, cuda=False)
    if results.shape[0] < n:
        raise ValueError("decompress_frames: results need nblocks entries")
    if dst_caps is not None:
        _arr(dst_caps, "decompress_frames dst_caps", torch.int32, cuda=False)
        if dst_caps.shape[0] < n:
            raise ValueError("decompress_frames: dst_caps need nblocks entries")
    elif n > 0 and dst.shape[1] != dst.stride(0):
        raise ValueError("decompress_frames: dst rows narrower than their stride need dst_caps")
    _on_cuda("decompress_frames", frames, offsets, dst, results, dst_caps)
    _check(lib().APE_LZ4_decompress_safe_frames_dev(_ptr(frames), _ptr(offsets), _ptr(dst),
                                                    dst.stride(0), _ptr(dst_caps), _ptr(results),
                                                    n, _stream(stream)),
           "APE_LZ4_decompress_safe_frames_dev")


# ---- socket path (include/ape_lz4_gpu.h, lz4_sock.hip; BASELINE config 5) ----
class RxBuf:
    """APE_LZ4_rxbuf: the receive buffer of ape_socket (ref src/ape_buffer.c:210-228),
    growable and registered for DMA, with the rewritten frame parser."""

    def __init__(self, initial=0):
        self._b = lib().APE_LZ4_rxbuf_new(initial)
        if not self._b:
            raise MemoryError("APE_LZ4_rxbuf_new")

    def prepare(self, more):
        return lib().APE_LZ4_rxbuf_prepare(self._b, more)

    def append(self, data):
        data = bytes(data)
        return lib().APE_LZ4_rxbuf_append(self._b, data, len(data))

    def frames(self, max_frames, max_block):
        """(n, offsets[0..n]) of the complete frames at the start, or (-1, []) if malformed."""
        off = (_C.c_longlong * (max_frames + 1))()
        n = lib().APE_LZ4_rxbuf_frames(self._b, off, max_frames, max_block)
        return n, (list(off[:n + 1]) if n >= 0 else [])

    def consume(self, n):
        lib().APE_LZ4_rxbuf_consume(self._b, n)

    def used(self):
        return lib().APE_LZ4_rxbuf_used(self._b)

    def room(self):
        return lib().APE_LZ4_rxbuf_room(self._b)

    def pinned(self):
        return bool(lib().APE_LZ4_rxbuf_pinned(self._b))

    def data(self):
        n = self.used()
        return _C.string_at(lib().APE_LZ4_rxbuf_data(self._b), n) if n else b""

    def free(self):
        if self._b:
            lib().APE_LZ4_rxbuf_free(self._b)
            self._b = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def socket_send_blocks(fd, src, block_size, batch):
    """APE_LZ4_socket_send_blocks: rows of src (uint8 numpy [N, S] or CPU tensor, S >=
    block_size) -> GPU encode -> framed stream written to fd.  Returns bytes written."""
    n = int(src.shape[0])
    stride = int(src.strides[0]) if hasattr(src, "strides") else int(src.stride(0))
    ptr = src.ctypes.data if hasattr(src, "ctypes") else src.data_ptr()
    r = lib().APE_LZ4_socket_send_blocks(fd, _C.c_void_p(ptr), stride, block_size, n, batch)
    if r < 0:
        raise GpuError("APE_LZ4_socket_send_blocks failed (%d): %s" % (r, gpu_last_error()))
    return r


def socket_recv_blocks(fd, dst, block_size, batch, results):
    """APE_LZ4_socket_recv_blocks: framed stream read from fd -> GPU decode -> rows of dst
    (uint8 numpy [N, S]); results (int32 numpy [N]) = decompress_safe results."""
    n = int(dst.shape[0])
    r = lib().APE_LZ4_socket_recv_blocks(fd, _C.c_void_p(dst.ctypes.data), int(dst.strides[0]),
                                         block_size, n, batch, _C.c_void_p(results.ctypes.data))
    if r < 0:
        raise GpuError("APE_LZ4_socket_recv_blocks failed (%d): %s" % (r, gpu_last_error()))
    return r


class Chain:
    """APE_LZ4_chain: nconn chained socket streams in the reference wire format (8 KiB
    chunks against the stream's last 64 KiB, [int32 size][block] frames; ref
    src/ape_socket.c:811-871, :1333-1467) with the GPU codec batched across connections."""

    def __init__(self, nconn, msg_len):
        self.nconn, self.msg_len = int(nconn), int(msg_len)
        self._c = lib().APE_LZ4_chain_new(self.nconn, self.msg_len)
        if not self._c:
            raise GpuError("APE_LZ4_chain_new failed: %s" % gpu_last_error())

    def _fds(self, fds):
        if len(fds) != self.nconn:
            raise ValueError("need %d fds" % self.nconn)
        return (_C.c_int * self.nconn)(*fds)

    def _rows(self, a, what):
        """The C side takes one stride: row pitch = nconn x strides[1], >= msg_len contiguous
        bytes per row."""
        import numpy as np
        if (not isinstance(a, np.ndarray) or a.dtype != np.uint8 or a.ndim != 3
                or a.shape[1] != self.nconn or a.shape[2] < self.msg_len or a.strides[2] != 1
                or a.strides[1] < self.msg_len or a.strides[0] != self.nconn * a.strides[1]):
            raise ValueError("%s: need a uint8 array [nmsg, %d, >= %d] with contiguous rows"
                             % (what, self.nconn, self.msg_len))

    def send(self, fds, msgs):
        """msgs: uint8 numpy [nmsg, nconn, S >= msg_len] (round m, connection i).  Returns the
        bytes written."""
        self._rows(msgs, "msgs")
        nmsg = int(msgs.shape[0])
        r = lib().APE_LZ4_chain_send(self._c, self._fds(fds), _C.c_void_p(msgs.ctypes.data),
                                     int(msgs.strides[1]), nmsg)
        if r < 0:
            raise GpuError("APE_LZ4_chain_send failed (%d): %s" % (r, gpu_last_error()))
        return r

    def recv(self, fds, out, status):
        """out: uint8 numpy [nmsg, nconn, S >= msg_len]; status: int32 numpy [nconn].  Returns
        the payload bytes (raises on a malformed stream or a failed decode)."""
        import numpy as np
        self._rows(out, "out")
        if (not isinstance(status, np.ndarray) or status.dtype != np.int32
                or status.shape != (self.nconn,) or not status.flags["C_CONTIGUOUS"]):
            raise ValueError("status: need a contiguous int32 array [%d]" % self.nconn)
        nmsg = int(out.shape[0])
        r = lib().APE_LZ4_chain_recv(self._c, self._fds(fds), _C.c_void_p(out.ctypes.data),
                                     int(out.strides[1]), nmsg, _C.c_void_p(status.ctypes.data))
        if r < 0:
            raise GpuError("APE_LZ4_chain_recv failed (%d): %s" % (r, gpu_last_error()))
        return r

    def free(self):
        if self._c:
            lib().APE_LZ4_chain_free(self._c)
            self._c = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


SOCKET_STATS = {"tx_h2d_ms": 0, "tx_encode_ms": 1, "tx_d2h_ms": 2, "tx_write_ms": 3,
                "tx_gpu_wait_ms": 4, "tx_batches": 5, "tx_total_ms": 6, "rx_total_ms": 7,
                "rx_read_ms": 8, "rx_parse_ms": 9, "rx_h2d_ms": 10, "rx_decode_ms": 11,
                "rx_d2h_ms": 12, "rx_gpu_wait_ms": 13, "rx_batches": 14, "rx_prepare_ms": 15}


def socket_stats(reset=True):
    """APE_LZ4_socket_stats: the time split of the socket calls since the last reset."""
    out = (_C.c_double * 16)()
    if lib().APE_LZ4_socket_stats(out, 1 if reset else 0) != 0:
        raise GpuError("APE_LZ4_socket_stats failed")
    return {k: round(out[i], 3) for k, i in SOCKET_STATS.items()}
