"""The master: experiment/trial lifecycle, searcher, scheduler, REST API (reference: ``master/``)."""

from determined_amd.master._core import Master
from determined_amd.master._server import MasterServer


def start_master(host: str = "127.0.0.1", port: int = 0, db_path: str = ":memory:", **kw) -> MasterServer:
    """Start an in-process master (tests, ``det deploy local``); returns the running server."""
    import socket

    if port == 0:
        with socket.socket() as s:
            s.bind((host, 0))
            port = s.getsockname()[1]
    m = Master(db_path=db_path, master_url=f"http://{host}:{port}", **kw)
    return MasterServer(m, host, port).start()
