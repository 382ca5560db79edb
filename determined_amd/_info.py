"""Information about the task a process runs in (reference: ``harness/determined/_info.py``).

The agent exports ``DET_*`` environment variables when it launches a task; ``get_cluster_info()``
returns ``None`` off-cluster, which makes ``core.init()`` fall back to local ("dummy") mode.
"""

import json
import os
from typing import Any, Dict, List, Optional


class TrialInfo:
    def __init__(self, trial_id: int, experiment_id: int, trial_seed: int, hparams: Dict[str, Any],
                 config: Dict[str, Any], steps_completed: int, trial_run_id: int, debug: bool = False) -> None:
        self.trial_id = trial_id
        self.experiment_id = experiment_id
        self.trial_seed = trial_seed
        self.hparams = hparams
        self._config = config
        self._steps_completed = steps_completed
        self._trial_run_id = trial_run_id
        self._debug = debug

    @classmethod
    def _from_env(cls) -> "TrialInfo":
        return cls(
            trial_id=int(os.environ["DET_TRIAL_ID"]),
            experiment_id=int(os.environ["DET_EXPERIMENT_ID"]),
            trial_seed=int(os.environ.get("DET_TRIAL_SEED", "0")),
            hparams=json.loads(os.environ.get("DET_HPARAMS", "{}")),
            config=json.loads(os.environ.get("DET_EXPERIMENT_CONFIG", "{}")),
            steps_completed=int(os.environ.get("DET_STEPS_COMPLETED", "0")),
            trial_run_id=int(os.environ.get("DET_TRIAL_RUN_ID", "0")),
            debug=os.environ.get("DET_DEBUG", "0") == "1",
        )


class ClusterInfo:
    def __init__(self, master_url: str, cluster_id: str, agent_id: str, slot_ids: List[int], task_id: str,
                 allocation_id: str, session_token: str, task_type: str, container_addrs: List[str],
                 container_rank: int, latest_checkpoint: Optional[str] = None,
                 trial: Optional[TrialInfo] = None) -> None:
        self.master_url = master_url
        self.cluster_id = cluster_id
        self.agent_id = agent_id
        self.slot_ids = slot_ids
        self.task_id = task_id
        self.allocation_id = allocation_id
        self.session_token = session_token
        self.task_type = task_type
        self.container_addrs = container_addrs
        self.container_rank = container_rank
        self._latest_checkpoint = latest_checkpoint
        self._trial = trial

    @property
    def latest_checkpoint(self) -> Optional[str]:
        return self._latest_checkpoint

    @property
    def trial(self) -> TrialInfo:
        if self._trial is None:
            raise RuntimeError("trial info is only available for TRIAL tasks")
        return self._trial

    @property
    def gpu_uuids(self) -> List[str]:
        return [str(s) for s in self.slot_ids] if os.environ.get("DET_USE_GPU", "0") == "1" else []

    @property
    def user_data(self) -> Dict[str, Any]:
        return self.trial._config.get("data", {}) if self._trial else {}

    @classmethod
    def _from_env(cls) -> Optional["ClusterInfo"]:
        if "DET_MASTER" not in os.environ or "DET_ALLOCATION_ID" not in os.environ:
            return None
        task_type = os.environ.get("DET_TASK_TYPE", "TRIAL")
        trial = TrialInfo._from_env() if task_type == "TRIAL" and "DET_TRIAL_ID" in os.environ else None
        return cls(
            master_url=os.environ["DET_MASTER"],
            cluster_id=os.environ.get("DET_CLUSTER_ID", "local"),
            agent_id=os.environ.get("DET_AGENT_ID", "agent"),
            slot_ids=json.loads(os.environ.get("DET_SLOT_IDS", "[]")),
            task_id=os.environ.get("DET_TASK_ID", ""),
            allocation_id=os.environ["DET_ALLOCATION_ID"],
            session_token=os.environ.get("DET_SESSION_TOKEN", ""),
            task_type=task_type,
            container_addrs=json.loads(os.environ.get("DET_CONTAINER_ADDRS", '["127.0.0.1"]')),
            container_rank=int(os.environ.get("DET_CONTAINER_RANK", "0")),
            latest_checkpoint=os.environ.get("DET_LATEST_CHECKPOINT") or None,
            trial=trial,
        )


def get_cluster_info() -> Optional[ClusterInfo]:
    return ClusterInfo._from_env()
