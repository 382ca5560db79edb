"""Single-GPU rehearsal of collective/compute interference: the headline bench with every DDP
bucket completion also launching a side-stream kernel that holds ``NBLK`` workgroups (one per
RCCL channel) for ``USEC`` microseconds -- the CU footprint of a bucket all-reduce on a multi-GPU
node.  ``DAMD_SIM_COLLECTIVE=NBLK:USEC[:end]``; ``end`` issues all of them after the backward
instead (the no-overlap alternative).  Prints the bench JSON line."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from determined_amd import ops  # noqa: E402
from determined_amd.parallel import ddp as D  # noqa: E402

spec = os.environ.get("DAMD_SIM_COLLECTIVE", "")
if spec:
    parts = spec.split(":")
    nblk, usec, at_end = int(parts[0]), float(parts[1]), len(parts) > 2 and parts[2] == "end"
    state = {"side": None, "n": 0}
    orig_complete, orig_finish = D.DistributedDataParallel._complete, D.DistributedDataParallel.finish

    def _occupy():
        if state["side"] is None:
            state["side"] = torch.cuda.Stream()
        state["side"].wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(state["side"]):
            ops.ext().occupy(nblk, usec)

    def _complete(self, b):
        orig_complete(self, b)
        if self._sync_enabled:
            if at_end:
                state["n"] += 1
            else:
                _occupy()

    def finish(self):
        for _ in range(state["n"]):
            _occupy()
        state["n"] = 0
        if state["side"] is not None:
            torch.cuda.current_stream().wait_stream(state["side"])
        orig_finish(self)

    D.DistributedDataParallel._complete = _complete
    D.DistributedDataParallel.finish = finish

if os.environ.get("DAMD_SIM_HIPRIO"):  # compute on a high-priority stream (collectives keep normal priority)
    hi = torch.cuda.Stream(device=int(os.environ.get("LOCAL_RANK", "0")), priority=-1)
    with torch.cuda.stream(hi):
        rc = bench.main()
    sys.exit(rc)
sys.exit(bench.main())
