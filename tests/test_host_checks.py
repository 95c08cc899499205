"""Host-side argument checks of the Python mirror that need no GPU: the RX input
must match the handle's in_dtype exactly, and a stream on another GPU is refused."""
import numpy as np
import pytest


def test_rx_input_dtype_and_shape(m):
    ok = m._check_rx_input(np.zeros((7, 2), np.float32), m.DTYPE_F32, "t")
    assert ok == 7
    assert m._check_rx_input(np.zeros((5, 2), np.float16), m.DTYPE_F16, "t") == 5
    assert m._check_rx_input(np.zeros(9, np.int16), m.DTYPE_I16, "t") == 9
    bad = [
        (np.zeros(9, np.int16), m.DTYPE_F32),          # i16 into an f32 handle: 2n bytes, not 8n
        (np.zeros(9, np.uint16), m.DTYPE_I16),         # uint16 is not int16
        (np.zeros((9, 2), np.int16), m.DTYPE_I16),     # i16 is (n,) real samples
        (np.zeros((9, 2), np.float16), m.DTYPE_F32),
        (np.zeros((9, 2), np.float32), m.DTYPE_F16),
        (np.zeros((9, 3), np.float32), m.DTYPE_F32),
        (np.zeros(18, np.float32), m.DTYPE_F32),
    ]
    for x, dt in bad:
        with pytest.raises(ValueError):
            m._check_rx_input(x, dt, "t")


def test_rx_input_torch_dtypes(m):
    torch = pytest.importorskip("torch")
    assert m._check_rx_input(torch.zeros((4, 2), dtype=torch.float32), m.DTYPE_F32, "t") == 4
    assert m._check_rx_input(torch.zeros(4, dtype=torch.int16), m.DTYPE_I16, "t") == 4
    with pytest.raises(ValueError):
        m._check_rx_input(torch.zeros(4, dtype=torch.int16), m.DTYPE_F32, "t")


def test_stream_of_another_device_refused(m):
    class FakeStream:
        device_index = 1
        cuda_stream = 1234
    assert m._stream_handle(FakeStream(), 1) == 1234
    with pytest.raises(ValueError):
        m._stream_handle(FakeStream(), 0)
