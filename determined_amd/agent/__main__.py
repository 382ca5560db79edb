"""``python -m determined_amd.agent --master-url http://127.0.0.1:8080``"""

import argparse
import logging
import os
import sys

from determined_amd.agent import Agent


def main(argv=None) -> int:
    p = argparse.ArgumentParser("determined_amd.agent")
    p.add_argument("--master-url", default=os.environ.get("DET_MASTER", "http://127.0.0.1:8080"))
    p.add_argument("--agent-id", default=None)
    p.add_argument("--slots", type=int, default=None, help="CPU slots (disables GPU detection)")
    p.add_argument("--gpus", default=None, help="comma-separated GPU ordinals to expose (default: all)")
    p.add_argument("--work-root", default=None)
    p.add_argument("--host", default=None, help="address other agents/ranks use to reach this node")
    p.add_argument("--label", default="")
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    gpus = [int(x) for x in a.gpus.split(",")] if a.gpus else None
    agent = Agent(a.master_url, a.agent_id, a.slots, gpus, a.work_root, a.host,
                  token=os.environ.get("DET_MASTER_TOKEN"), label=a.label)
    try:
        agent.run()
    except KeyboardInterrupt:
        agent.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
