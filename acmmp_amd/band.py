"""Row-band split of ONE RunPatchMatch over the ranks of a process group
(SURVEY §5 "image-size scaling" / cfg5's "tiled per-image"; the reference has
no intra-image split): every rank runs acmmp_run_patchmatch_band on the same
inputs with its own rows, the halo rows the far searches read (23 rows:
3 + 2 * 10, src/ACMMP.cu:819-826) travel between neighbouring bands after
every half-sweep, and the bands are gathered afterwards. Results are
bit-identical to the unsplit run (tests/test_gpu_band.py).

The exchange runs on torch.distributed: RCCL (nccl backend) on device
buffers between GPUs, or gloo through host memory (several ranks sharing one
GPU in the tests).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _abi
from .engine import AcmmpError


def bands(height: int, n: int) -> list:
    """n contiguous row bands [lo, hi) tiling 0..height, sizes differing by at
    most one row; every band must hold the halo (a neighbour two bands away
    is never read)."""
    if n < 1 or height < n * _abi.BAND_HALO:
        raise AcmmpError(f"{height} rows cannot be split into {n} bands of >= {_abi.BAND_HALO} rows")
    base, extra = divmod(height, n)
    out, lo = [], 0
    for k in range(n):
        hi = lo + base + (1 if k < extra else 0)
        out.append((lo, hi))
        lo = hi
    return out


class _DeviceArray:
    """A device allocation seen by torch (__cuda_array_interface__)."""

    def __init__(self, ptr: int, n: int, typestr: str):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (int(ptr), False),
                                         "version": 2, "strides": None}


def device_view(ptr: int, n: int, dtype: torch.dtype, device: torch.device) -> torch.Tensor:
    typestr = {torch.float32: "<f4", torch.int32: "<i4"}[dtype]
    return torch.as_tensor(_DeviceArray(ptr, n, typestr), device=device)


class TorchBandExchange:
    """The halo exchange of one participant: `members` are the global ranks
    of the bands in row order, `index` this rank's position among them.
    `comm_device` is where the collective runs (cuda: RCCL; cpu: gloo)."""

    def __init__(self, members: list, index: int, device: torch.device, comm_device: torch.device, group=None):
        self.members = members
        self.index = index
        self.device = device
        self.comm_device = comm_device
        self.group = group
        self.exchanges = 0

    def __call__(self, halo: _abi.BandHalo):
        Wh = int(halo.Wh)
        rows = max(halo.recv_down_hi, halo.send_down_hi, halo.recv_up_hi, halo.send_up_hi)
        # the sweep that wrote these rows ran on the engine's stream
        torch.cuda.ExternalStream(int(halo.stream), device=self.device).synchronize()
        plane = device_view(halo.plane, rows * Wh * 4, torch.float32, self.device).view(rows, Wh * 4)
        cost = device_view(halo.cost, rows * Wh, torch.float32, self.device).view(rows, Wh)
        sv = device_view(halo.sv, rows * Wh, torch.int32, self.device).view(rows, Wh)

        def pack(lo, hi):
            return torch.cat([plane[lo:hi].reshape(-1), cost[lo:hi].reshape(-1),
                              sv[lo:hi].view(torch.float32).reshape(-1)]).to(self.comm_device)

        def unpack(buf, lo, hi):
            n = (hi - lo) * Wh
            buf = buf.to(self.device)
            plane[lo:hi] = buf[:4 * n].view(hi - lo, Wh * 4)
            cost[lo:hi] = buf[4 * n:5 * n].view(hi - lo, Wh)
            sv[lo:hi] = buf[5 * n:].view(torch.int32).view(hi - lo, Wh)

        ops, recvs = [], []
        for peer_off, (slo, shi), (rlo, rhi) in ((-1, (halo.send_up_lo, halo.send_up_hi),
                                                  (halo.recv_up_lo, halo.recv_up_hi)),
                                                 (1, (halo.send_down_lo, halo.send_down_hi),
                                                  (halo.recv_down_lo, halo.recv_down_hi))):
            k = self.index + peer_off
            if not (0 <= k < len(self.members)):
                continue
            peer = self.members[k]
            if shi > slo:
                ops.append(dist.P2POp(dist.isend, pack(slo, shi), peer, self.group))
            if rhi > rlo:
                buf = torch.empty(((rhi - rlo) * Wh * 6,), dtype=torch.float32, device=self.comm_device)
                ops.append(dist.P2POp(dist.irecv, buf, peer, self.group))
                recvs.append((buf, rlo, rhi))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        for buf, lo, hi in recvs:
            unpack(buf, lo, hi)
        # the engine's next sweep does not wait on torch's stream
        torch.cuda.current_stream(self.device).synchronize()
        self.exchanges += 1


def gather_bands(planes: torch.Tensor, costs: torch.Tensor, bands_: list, members: list, index: int,
                 comm_device: torch.device, group=None):
    """Every band's rows of (H, W, 4) planes and (H, W) costs from its rank,
    assembled in place on every participant. The assembly is enqueued on
    torch's current stream (through gloo: pinned staging buffers and
    asynchronous host-to-device copies); an engine reading the result orders
    its stream after torch's first (ACMMP._after_producer)."""
    if len(members) == 1:
        return planes, costs
    H, W = costs.shape
    rmax = max(hi - lo for lo, hi in bands_)
    lo, hi = bands_[index]
    send = torch.zeros((rmax, W, 5), dtype=torch.float32, device=comm_device)
    send[:hi - lo, :, :4] = planes[lo:hi].to(comm_device)
    send[:hi - lo, :, 4] = costs[lo:hi].to(comm_device)
    pin = comm_device.type == "cpu" and planes.is_cuda
    recv = [torch.empty(send.shape, dtype=send.dtype, device=comm_device, pin_memory=pin) for _ in members]
    dist.all_gather(recv, send, group=group)
    for k, (blo, bhi) in enumerate(bands_):
        if k == index:
            continue
        r = recv[k].to(planes.device, non_blocking=True)
        planes[blo:bhi] = r[:bhi - blo, :, :4]
        costs[blo:bhi] = r[:bhi - blo, :, 4]
    return planes, costs


def run_split(eng, bands_: list, members: list, index: int, device: torch.device, comm_device: torch.device,
              group=None, planar_prior: bool = False):
    """One ProcessProblem's RunPatchMatch (and, with planar_prior, the
    prior construction and second run of src/acmmp_definitions.cpp:306-379)
    split into row bands; returns the full (planes, costs) on every rank."""
    lo, hi = bands_[index]
    ex = TorchBandExchange(members, index, device, comm_device, group)
    W, H = eng.size
    planes = torch.empty((H, W, 4), dtype=torch.float32, device=device)
    costs = torch.empty((H, W), dtype=torch.float32, device=device)
    for run in range(2 if planar_prior else 1):
        eng.run_band(lo, hi, ex)
        eng.export_results(planes.data_ptr(), costs.data_ptr(), 0)
        eng.synchronize()
        gather_bands(planes, costs, bands_, members, index, comm_device, group)
        if planar_prior and run == 0:
            # support points + Delaunay need the whole image: every rank
            # builds the same prior from the gathered state (the engine's
            # copy waits for the assembly on torch's stream)
            eng.set_plane_hypotheses_device(planes.data_ptr(), costs.data_ptr())
            eng.prepare_planar_prior()
    return planes, costs
