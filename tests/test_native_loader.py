"""Native C++ token loader (csrc/runtime/token_loader.cpp): windows of a memory-mapped corpus or
synthetic ids, deterministic per (seed, rank, batch) whatever the worker-thread count."""
import os
import tempfile

import numpy as np
import pytest
import torch

from trustworthy_dl.runtime import native

pytestmark = pytest.mark.skipif(not native.available(), reason="libtdl_runtime.so not built")


def _take(loader, n):
    out = []
    for _ in range(n):
        b = loader.next_batch()
        out.append((b["input"].clone(), b["target"].clone(), b["batch_index"]))
    return out


def test_synthetic_stream_is_deterministic_across_thread_counts():
    a = native.NativeTokenLoader(8, 64, seed=7, threads=1, slots=3)
    b = native.NativeTokenLoader(8, 64, seed=7, threads=4, slots=6)
    ra, rb = _take(a, 12), _take(b, 12)
    for (ia, ta, ka), (ib, tb, kb) in zip(ra, rb):
        assert ka == kb
        assert torch.equal(ia, ib) and torch.equal(ta, tb)
        assert torch.equal(ia[:, 1:], ta[:, :-1])          # next-token targets
        assert int(ia.min()) >= 0 and int(ia.max()) < 50257
    assert [k for _, _, k in ra] == list(range(12))
    a.close()
    b.close()


def test_ranks_read_distinct_batches():
    r0 = native.NativeTokenLoader(4, 32, seed=1, rank=0, world=2)
    r1 = native.NativeTokenLoader(4, 32, seed=1, rank=1, world=2)
    x0, x1 = r0.next_batch()["input"].clone(), r1.next_batch()["input"].clone()
    assert not torch.equal(x0, x1)


@pytest.mark.parametrize("token_bytes,dtype", [(2, np.uint16), (4, np.uint32)])
def test_memory_mapped_corpus_windows(token_bytes, dtype):
    corpus = (np.arange(10_000, dtype=np.int64) * 7 % 50_000).astype(dtype)
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "tokens.bin")
        corpus.tofile(path)
        L = native.NativeTokenLoader(6, 33, path=path, token_bytes=token_bytes, seed=3, threads=2)
        assert L.num_tokens == 10_000
        ref = corpus.astype(np.int64)
        for _ in range(5):
            b = L.next_batch()
            for row_in, row_tg in zip(b["input"].numpy(), b["target"].numpy()):
                # every row is a contiguous window of the corpus, target shifted by one
                start = int(np.flatnonzero(ref == row_in[0])[0]) if (ref == row_in[0]).any() else -1
                assert start >= 0
                starts = np.flatnonzero(ref[:len(ref) - 33] == row_in[0])
                assert any(np.array_equal(ref[s:s + 33], row_in) and np.array_equal(ref[s + 1:s + 34], row_tg)
                           for s in starts)
        L.close()


def test_iterable_protocol_and_count():
    L = native.NativeTokenLoader(2, 8, seed=0, num_batches=5)
    n = sum(1 for _ in L)
    assert n == 5
    L.close()
