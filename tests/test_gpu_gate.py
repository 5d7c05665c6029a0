"""The multi-GPU pipeline's encode gate (runtime.EncodeGate: one signal word,
hipStreamWriteValue32 / hipStreamWaitValue32): a stream waiting at a yield
point does not pass while the gate is held, and passes once it is released;
`yield_point` waits only on the gated stream."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda")


def test_gate_orders_waiter_after_release(dev):
    from aligned_vggt.runtime import EncodeGate, dedicated_stream
    gate = EncodeGate(dev)
    a, b = dedicated_stream(dev), dedicated_stream(dev)
    x = torch.zeros(1, device=dev)
    y = torch.full((1,), -1.0, device=dev)
    torch.cuda.synchronize()
    with torch.cuda.stream(a):
        gate.begin(a)
        held = torch.cuda.Event()
        held.record(a)
        torch.cuda._sleep(50_000_000)  # ~20 ms of spinning on stream a while the gate is held
        x.fill_(1.0)
        gate.end(a)
    with torch.cuda.stream(b):
        b.wait_event(held)  # the gate is 1 when b reaches its wait
        gate.wait(b.cuda_stream)
        y.copy_(x)
    torch.cuda.synchronize()
    assert y.item() == 1.0  # b's copy ran after a's fill: it waited for the release
    # released gate: a wait passes at once
    with torch.cuda.stream(b):
        gate.wait(b.cuda_stream)
        y.fill_(2.0)
    torch.cuda.synchronize()
    assert y.item() == 2.0
    gate.close()


def test_yield_point_only_on_gated_stream(dev, monkeypatch):
    from aligned_vggt import runtime as R
    gate = R.EncodeGate(dev)
    enc, other = R.dedicated_stream(dev), R.dedicated_stream(dev)
    calls = []
    monkeypatch.setattr(gate, "wait", lambda handle: calls.append(handle))
    with R.gated(enc, gate):
        with torch.cuda.stream(enc):
            R.yield_point()
        with torch.cuda.stream(other):
            R.yield_point()
    R.yield_point()  # outside: no gate
    assert calls == [enc.cuda_stream]
    gate.close()
