"""CPU: the native generator (blockgen.h via libjfsgpu) equals the Python spec."""
import ctypes

import pytest

from juicefs_amd.blockgen import gen_block


@pytest.mark.parametrize("cls", ["T", "Z", "R"])
@pytest.mark.parametrize("n", [0, 1, 7, 100, 4096, 100003])
def test_native_generator_matches_python(lib, cls, n):
    buf = ctypes.create_string_buffer(max(n, 1))
    lib.jfs_gen_block_host(buf, n, cls.encode(), 4242 + n)
    assert buf.raw[:n] == gen_block(cls, 4242 + n, n)


def test_text_block_is_text_like():
    b = gen_block("T", 5, 200000)
    assert b.count(b" ") > 20000 and b.count(b"\n") >= 40
