"""What the first 8-GPU record relies on, checked on the one-GPU box:
* HIP IPC between two fresh processes under the environment bench.py gives its ranks
  (HSA_ENABLE_IPC_MODE_LEGACY=0): the mechanism RCCL's P2P/IPC transport maps a peer's buffers with;
* chr_comm_info: what RCCL's communicator reports (ncclCommCount, ncclCommUserRank, ncclCommCuDevice)
  and the device's PCI bus id, the fields of the N>1 line's `rccl` record."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
PROBE = os.path.join(HERE, "ipc_probe.py")


def _env():
    env = dict(os.environ)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    return env


@pytest.mark.parametrize("nbytes", [4096, 8 << 20])
def test_hip_ipc_handle_between_two_processes(nbytes):
    owner = subprocess.Popen([sys.executable, PROBE, "owner", str(nbytes)], stdin=subprocess.PIPE,
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=_env())
    try:
        handle = owner.stdout.readline().strip()
        assert len(handle) == 128, (handle, owner.stderr.read() if owner.poll() is not None else "")
        peer = subprocess.run([sys.executable, PROBE, "peer", handle, str(nbytes)], capture_output=True, text=True,
                              env=_env(), timeout=120)
        assert peer.returncode == 0 and peer.stdout.strip().endswith("OK"), (peer.stdout, peer.stderr[-2000:])
        owner.stdin.write("done\n")
        owner.stdin.flush()
        out, err = owner.communicate(timeout=120)
        assert owner.returncode == 0 and out.strip().endswith("OK"), (out, err[-2000:])
    finally:
        if owner.poll() is None:
            owner.kill()
            owner.wait()


def test_comm_info_reports_rccl_view():
    sys.path[:0] = [os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")]
    import torch

    import chiara_amd as ca

    comm = ca.Comm(1, ca.get_unique_id(), 0, 0)
    try:
        info = comm.info()
        assert info["nranks"] == 1 and info["rank"] == 0 and info["device"] == 0
        bus = info["pci_bus_id"]
        props = torch.cuda.get_device_properties(0)
        # "dddd:bb:dd.f" with the bus number torch reports for the same device
        assert len(bus.split(":")) == 3 and int(bus.split(":")[1], 16) == props.pci_bus_id, (bus, props.pci_bus_id)
    finally:
        comm.destroy()
