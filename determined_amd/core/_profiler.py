"""System-metrics profiler (reference: ``harness/determined/core/_profiler.py``, which uses pynvml).

Samples CPU, memory, disk, network (psutil) and AMD GPU utilisation / VRAM / power straight
from the amdgpu sysfs interface (``/sys/class/drm/card*/device``), so it needs no vendor Python
bindings.  A collector thread samples every ``sampling_interval`` seconds and a shipper thread
reports the averaged groups to the master as ``profiling`` metrics.
"""

import glob
import logging
import os
import queue
import threading
import time
from typing import Any, Dict, List, Optional

logger = logging.getLogger("determined_amd.core")


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def amd_gpus() -> List[str]:
    """Device directories of amdgpu cards (those exposing gpu_busy_percent)."""
    out = []
    for d in sorted(glob.glob("/sys/class/drm/card*/device")):
        if os.path.exists(os.path.join(d, "gpu_busy_percent")):
            out.append(d)
    return out


def sample_gpus() -> Dict[str, Dict[str, float]]:
    res: Dict[str, Dict[str, float]] = {}
    for i, d in enumerate(amd_gpus()):
        m: Dict[str, float] = {}
        busy = _read(os.path.join(d, "gpu_busy_percent"))
        if busy is not None:
            m["gpu_util"] = float(busy) / 100.0
        used = _read(os.path.join(d, "mem_info_vram_used"))
        total = _read(os.path.join(d, "mem_info_vram_total"))
        if used is not None:
            m["gpu_free_memory"] = float(total) - float(used) if total else 0.0
            m["gpu_used_memory"] = float(used)
        power = glob.glob(os.path.join(d, "hwmon", "hwmon*", "power1_average"))
        if power:
            p = _read(power[0])
            if p is not None:
                m["gpu_power_w"] = float(p) / 1e6
        res[str(i)] = m
    return res


class _Collector(threading.Thread):
    def __init__(self, interval: float, per_report: int, out: "queue.Queue") -> None:
        super().__init__(daemon=True, name="profiler-collector")
        self.interval = interval
        self.per_report = per_report
        self.out = out
        self._stop = threading.Event()

    def run(self) -> None:
        import psutil

        samples: List[Dict[str, Any]] = []
        last_net = psutil.net_io_counters()
        last_disk = psutil.disk_io_counters()
        last_t = time.time()
        while not self._stop.wait(self.interval):
            now = time.time()
            dt = max(now - last_t, 1e-6)
            net = psutil.net_io_counters()
            disk = psutil.disk_io_counters()
            s: Dict[str, Any] = {
                "cpu": {"cpu_util_simple": psutil.cpu_percent() / 100.0},
                "memory": {"memory_free": float(psutil.virtual_memory().available)},
                "network": {
                    "net_throughput_sent": (net.bytes_sent - last_net.bytes_sent) / dt,
                    "net_throughput_recv": (net.bytes_recv - last_net.bytes_recv) / dt,
                },
            }
            if disk is not None and last_disk is not None:
                s["disk"] = {
                    "disk_throughput_read": (disk.read_bytes - last_disk.read_bytes) / dt,
                    "disk_throughput_write": (disk.write_bytes - last_disk.write_bytes) / dt,
                    "disk_iops": (disk.read_count + disk.write_count - last_disk.read_count
                                  - last_disk.write_count) / dt,
                }
            s["gpu"] = sample_gpus()
            last_net, last_disk, last_t = net, disk, now
            samples.append(s)
            if len(samples) >= self.per_report:
                self.out.put(_average(samples))
                samples = []

    def stop(self) -> None:
        self._stop.set()


def _average(samples: List[Dict[str, Any]]) -> Dict[str, Any]:
    """Average nested numeric dicts (depth <= 2)."""
    out: Dict[str, Any] = {}
    for s in samples:
        for g, vals in s.items():
            dst = out.setdefault(g, {})
            for k, v in vals.items():
                if isinstance(v, dict):
                    d2 = dst.setdefault(k, {})
                    for k2, v2 in v.items():
                        d2[k2] = d2.get(k2, 0.0) + v2 / len(samples)
                else:
                    dst[k] = dst.get(k, 0.0) + v / len(samples)
    return out


class ProfilerContext:
    def __init__(self, session: Any = None, agent_id: str = "", trial_id: int = 0, run_id: int = 0,
                 distributed: Any = None) -> None:
        self._session = session
        self._agent_id = agent_id
        self._trial_id = trial_id
        self._run_id = run_id
        self._dist = distributed
        self._collector: Optional[_Collector] = None
        self._shipper: Optional[threading.Thread] = None
        self._q: "queue.Queue" = queue.Queue()
        self._step = 0

    def on(self, sampling_interval: int = 1, samples_per_report: int = 10) -> None:
        if self._collector is not None:
            return
        if self._dist is not None and self._dist.local_rank != 0:
            return  # one sampler per node
        self._collector = _Collector(float(sampling_interval), samples_per_report, self._q)
        self._collector.start()
        self._shipper = threading.Thread(target=self._ship, daemon=True, name="profiler-shipper")
        self._shipper.start()

    def _ship(self) -> None:
        while True:
            item = self._q.get()
            if item is None:
                return
            self._step += 1
            for group, vals in item.items():
                try:
                    self._report(group, vals)
                except Exception as e:
                    logger.debug(f"profiler ship failed: {e}")

    def _report(self, group: str, vals: Dict[str, Any]) -> None:
        if self._session is None:
            return
        flat: Dict[str, Any] = {}
        for k, v in vals.items():
            if isinstance(v, dict):
                for k2, v2 in v.items():
                    flat[f"{k}/{k2}"] = v2
            else:
                flat[k] = v
        self._session.post(f"/api/v1/trials/{self._trial_id}/metrics", {
            "group": f"profiling_{group}", "steps_completed": self._step, "trial_run_id": self._run_id,
            "metrics": {**flat, "agent_id": self._agent_id}})

    def off(self) -> None:
        if self._collector is not None:
            self._collector.stop()
            self._collector = None
            self._q.put(None)

    def _close(self) -> None:
        self.off()


class DummyProfilerContext(ProfilerContext):
    def __init__(self) -> None:
        super().__init__()

    def on(self, sampling_interval: int = 1, samples_per_report: int = 10) -> None:
        pass

    def off(self) -> None:
        pass
