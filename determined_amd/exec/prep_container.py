"""Pre-launch checks for a task's process tree (reference: ``harness/determined/exec/prep_container.py``).

The reference runs this inside each Docker container before the entrypoint: download the
model definition, rendezvous with the other containers, register a proxy address and tell the
master the container is up.  Our agent launches process groups directly on the MI355X node, so
what remains is:

* ``--resources``: verify the GPUs this task was given are really there (KFD topology in sysfs,
  read WITHOUT initialising HIP -- the launcher must stay exec-safe) and report their HBM size;
* ``--rendezvous``: materialise the rendezvous info (chief address, node rank, slots per node)
  that the master put into ``DET_*`` variables as ``$DET_RENDEZVOUS_FILE`` (JSON) for launch
  layers that read a file, and pick the network interface RCCL's bootstrap should use when the
  gang spans nodes (``NCCL_SOCKET_IFNAME``);
* ``--download-context``: fetch the experiment's model definition into the working directory.
"""

import argparse
import base64
import io
import json
import os
import pathlib
import socket
import sys
import tarfile
from typing import Any, Dict, List, Optional

KFD_NODES = pathlib.Path("/sys/class/kfd/kfd/topology/nodes")


def _kv(path: pathlib.Path) -> Dict[str, str]:
    out: Dict[str, str] = {}
    try:
        for line in path.read_text().splitlines():
            parts = line.split()
            if len(parts) == 2:
                out[parts[0]] = parts[1]
    except OSError:
        pass
    return out


def gpu_inventory(root: pathlib.Path = KFD_NODES) -> List[Dict[str, Any]]:
    """One entry per GPU KFD node: ``{index, gfx_target_version, simd_count, hbm_bytes}``."""
    gpus: List[Dict[str, Any]] = []
    if not root.exists():
        return gpus
    for node in sorted(root.iterdir(), key=lambda p: int(p.name) if p.name.isdigit() else 1 << 30):
        props = _kv(node / "properties")
        if int(props.get("simd_count", "0")) <= 0:
            continue
        hbm = 0
        for bank in sorted((node / "mem_banks").glob("*")):
            hbm += int(_kv(bank / "properties").get("size_in_bytes", "0"))
        gpus.append({"index": len(gpus), "gfx_target_version": int(props.get("gfx_target_version", "0")),
                     "simd_count": int(props["simd_count"]), "hbm_bytes": hbm})
    return gpus


def check_resources(slot_ids: List[int], use_gpu: bool, root: pathlib.Path = KFD_NODES) -> List[Dict[str, Any]]:
    """Raise if a slot this task was given is not a visible GPU; return the matched GPUs."""
    if not use_gpu:
        return []
    inv = gpu_inventory(root)
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis:
        allowed = [int(x) for x in vis.split(",") if x.strip().isdigit()]
        if len(allowed) < len(slot_ids):
            raise RuntimeError(f"task was given {len(slot_ids)} slots but only {len(allowed)} GPUs are visible "
                               f"(HIP_VISIBLE_DEVICES={vis})")
    by_idx = {g["index"]: g for g in inv}
    missing = [s for s in slot_ids if s not in by_idx]
    if inv and missing:
        raise RuntimeError(f"slots {missing} are not GPUs on this node (found {len(inv)} GPUs)")
    return [by_idx[s] for s in slot_ids if s in by_idx]


def rendezvous_info(env: Optional[Dict[str, str]] = None) -> Dict[str, Any]:
    env = dict(os.environ if env is None else env)
    addrs = json.loads(env.get("DET_CONTAINER_ADDRS", '["127.0.0.1"]'))
    rank = int(env.get("DET_CONTAINER_RANK", "0"))
    slots = json.loads(env.get("DET_SLOT_IDS", "[0]"))
    return {"addrs": addrs, "rank": rank, "chief": addrs[0] if addrs else "127.0.0.1",
            "num_nodes": len(addrs), "slots_per_node": len(slots)}


def interface_for(addr: str) -> Optional[str]:
    """The local interface whose IPv4 address equals ``addr`` (None for loopback / not found)."""
    if addr.startswith("127."):
        return "lo"
    try:
        import psutil
    except ImportError:  # pragma: no cover
        return None
    for name, snics in psutil.net_if_addrs().items():
        for s in snics:
            if s.family == socket.AF_INET and s.address == addr:
                return name
    return None


def do_rendezvous(path: str, env: Optional[Dict[str, str]] = None) -> Dict[str, Any]:
    info = rendezvous_info(env)
    if info["num_nodes"] > 1:
        me = info["addrs"][info["rank"]]
        iface = interface_for(me)
        if iface:
            info["socket_ifname"] = iface
    with open(path, "w") as f:
        json.dump(info, f)
    return info


def download_context(tgz_b64: str, dest: str) -> None:
    with tarfile.open(fileobj=io.BytesIO(base64.b64decode(tgz_b64)), mode="r:gz") as tf:
        tf.extractall(dest, filter="data")


def main(argv: List[str]) -> int:
    ap = argparse.ArgumentParser(prog="prep_container")
    ap.add_argument("--resources", action="store_true")
    ap.add_argument("--rendezvous", action="store_true")
    ap.add_argument("--download-context", action="store_true")
    ap.add_argument("--trial", action="store_true", help="accepted for compatibility; implied by DET_TRIAL_ID")
    a = ap.parse_args(argv)
    out: Dict[str, Any] = {}
    if a.resources:
        slots = json.loads(os.environ.get("DET_SLOT_IDS", "[]"))
        out["gpus"] = check_resources(slots, os.environ.get("DET_USE_GPU", "0") == "1")
    if a.rendezvous:
        path = os.environ.get("DET_RENDEZVOUS_FILE", os.path.join(os.getcwd(), ".det_rendezvous.json"))
        out["rendezvous"] = do_rendezvous(path)
    if a.download_context:
        from determined_amd.common.api import Session

        eid = os.environ["DET_EXPERIMENT_ID"]
        sess = Session(os.environ["DET_MASTER"], token=os.environ.get("DET_SESSION_TOKEN") or None)
        download_context(sess.get(f"/api/v1/experiments/{eid}/model_def")["b64_tgz"], os.getcwd())
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
