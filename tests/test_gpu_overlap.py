"""Cross-bucket overlap: bucket i+1's top-k step on a second stream waits only for
bucket i's main pass (ops.MainEvent, grace_topk_arm_main_event / grace_stream_wait_event), so its
bracket runs beside bucket i's finalize.  Results must equal a serial run on one stream bit for
bit (per-stream workspaces, per-name step order kept)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1 << 22, (1 << 21) + 37])
def test_two_stream_main_event_steps_equal_serial(n):
    from grace_amd.dist.communicator.allgather import Allgather
    from grace_amd.dist.compressor.topk import TopKCompressor
    from grace_amd.dist.memory.residual import ResidualMemory
    from grace_amd.ops import MainEvent

    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    grads = []
    for j in range(4):
        gen.manual_seed(100 + j)
        grads.append(torch.randn(n, device=dev, generator=gen))
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
    evs = [MainEvent(), MainEvent()]
    ovl = Allgather(TopKCompressor(0.01), ResidualMemory(), 1)
    ser = Allgather(TopKCompressor(0.01), ResidualMemory(), 1)
    outs = []
    for i in range(12):
        j = i % 4
        st = streams[j % 2]
        with torch.cuda.stream(st):
            if i > 0:
                evs[(i - 1) % 2].wait(st)
            evs[i % 2].arm()
            outs.append(ovl.step(grads[j], f"b{j}").clone())
    torch.cuda.synchronize()
    for i in range(12):
        j = i % 4
        ref = ser.step(grads[j], f"b{j}")
        assert torch.equal(outs[i], ref), f"step {i}"
    for j in range(4):
        assert torch.equal(ovl.memory.residuals[f"b{j}"], ser.memory.residuals[f"b{j}"])
