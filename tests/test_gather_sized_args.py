"""CPU: sbecodec.gather_encoded_sized refuses, before anything reaches the C ABI, the arguments
that would leave a rank blocked in RCCL or let RCCL read / write past a tensor:
zero capacities on any rank, root capacities larger than dst / dst_off, shard buffers smaller
than this rank's planned sizes.  No device and no library are needed: every check runs first."""
import types

import pytest
import torch

import sbecodec


@pytest.fixture
def host_tensors(monkeypatch):
    # the device-tensor check (_dev) is the only thing between the arguments and the size checks;
    # let CPU tensors through it, and make any call into the library a test failure
    monkeypatch.setattr(sbecodec, "_dev", lambda t, dtype, name: t)

    def no_lib():
        raise AssertionError("the C ABI was reached")

    monkeypatch.setattr(sbecodec, "lib", no_lib)


def comm(world, rank):
    return types.SimpleNamespace(world=world, rank=rank, _h=None)


SIZES = [(256 * 10, 10), (256 * 7, 7)]


def bufs(nbytes, noff):
    return torch.empty(nbytes, dtype=torch.uint8), torch.empty(noff, dtype=torch.int64)


@pytest.mark.parametrize("rank", [0, 1])
@pytest.mark.parametrize("caps", [(0, 0), (0, 18), (4352, 0)])
def test_zero_capacities_refused_on_every_rank(host_tensors, rank, caps):
    out, off = bufs(*SIZES[rank])
    dst, dst_off = bufs(4352, 18) if rank == 0 else (None, None)
    with pytest.raises(sbecodec.SbeError, match="capacit"):
        sbecodec.gather_encoded_sized(comm(2, rank), SIZES, out, off, root=0, dst=dst, dst_off=dst_off,
                                      dst_capacity=caps[0], dst_off_capacity=caps[1])


@pytest.mark.parametrize("caps", [(4353, 18), (4352, 19)])
def test_root_capacities_past_its_tensors_refused(host_tensors, caps):
    out, off = bufs(*SIZES[0])
    dst, dst_off = bufs(4352, 18)
    with pytest.raises(sbecodec.SbeError, match="exceed"):
        sbecodec.gather_encoded_sized(comm(2, 0), SIZES, out, off, root=0, dst=dst, dst_off=dst_off,
                                      dst_capacity=caps[0], dst_off_capacity=caps[1])


@pytest.mark.parametrize("rank", [0, 1])
@pytest.mark.parametrize("short", ["bytes", "offsets"])
def test_shard_smaller_than_its_planned_size_refused(host_tensors, rank, short):
    b, m = SIZES[rank]
    out, off = bufs(b - 1 if short == "bytes" else b, m - 1 if short == "offsets" else m)
    dst, dst_off = bufs(4352, 18) if rank == 0 else (None, None)
    with pytest.raises(sbecodec.SbeError, match="shard buffers"):
        sbecodec.gather_encoded_sized(comm(2, rank), SIZES, out, off, root=0, dst=dst, dst_off=dst_off,
                                      dst_capacity=4352, dst_off_capacity=18)


def test_valid_arguments_reach_the_library(host_tensors):
    out, off = bufs(*SIZES[1])
    with pytest.raises(AssertionError, match="C ABI was reached"):
        sbecodec.gather_encoded_sized(comm(2, 1), SIZES, out, off, root=0, dst_capacity=4352, dst_off_capacity=18)
