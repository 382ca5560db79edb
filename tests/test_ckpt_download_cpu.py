"""Checkpoint download modes (reference ``common/experimental/checkpoint/_checkpoint.py``: DIRECT / MASTER /
AUTO): the master streams a tar.gz of the checkpoint for clients without storage access."""

import pytest


@pytest.fixture()
def ckpt(tmp_path):
    from determined_amd.experimental import client, core_v2
    from determined_amd.master import start_master

    srv = start_master()
    url = f"http://127.0.0.1:{srv.port}"
    ctx = core_v2.init_context(defaults=core_v2.DefaultConfig(
        name="dl", checkpoint_storage={"type": "shared_fs", "host_path": str(tmp_path / "store")}), master=url)
    with ctx:
        with ctx.checkpoint.store_path({"steps_completed": 1}) as (path, uuid):
            (path / "weights.bin").write_bytes(b"\x00\x01" * 1000)
            (path / "sub").mkdir()
            (path / "sub" / "cfg.json").write_text('{"a": 1}')
    client.login(url)
    yield client, client.get_checkpoint(uuid), tmp_path
    srv.stop()
    srv.master.close()


def _check(d):
    import pathlib

    d = pathlib.Path(d)
    assert (d / "weights.bin").read_bytes() == b"\x00\x01" * 1000
    assert (d / "sub" / "cfg.json").read_text() == '{"a": 1}'
    assert (d / "metadata.json").exists()


def test_direct_and_master_download(ckpt):
    client, ck, tmp = ckpt
    _check(ck.download(str(tmp / "direct"), mode=client.DownloadMode.DIRECT))
    _check(ck.download(str(tmp / "via_master"), mode=client.DownloadMode.MASTER))


def test_auto_falls_back_to_the_master(ckpt, monkeypatch):
    client, ck, tmp = ckpt

    def no_access(self, path):
        raise FileNotFoundError("storage not mounted here")

    monkeypatch.setattr(type(ck), "_download_direct", no_access)
    _check(ck.download(str(tmp / "auto"), mode=client.DownloadMode.AUTO))
    with pytest.raises(FileNotFoundError):
        ck.download(str(tmp / "direct_only"), mode=client.DownloadMode.DIRECT)


def test_master_download_of_unknown_checkpoint_fails(ckpt):
    import requests

    client, ck, tmp = ckpt
    r = requests.get(f"{ck._session.master_url}/api/v1/checkpoints/00000000-0000-0000-0000-000000000000/download")
    assert r.status_code == 404
