"""Object-store checkpoint storage over the stores' plain HTTP APIs (reference:
``harness/determined/common/storage/{s3,gcs,azure}.py``, which wrap boto3 / google-cloud-storage /
azure-storage-blob -- none of them are installed here, so the requests are built directly):

* :class:`S3StorageManager` -- S3 REST with AWS Signature V4 (``UNSIGNED-PAYLOAD`` bodies, so
  multi-GB checkpoint files stream from disk), path-style addressing when ``endpoint_url`` is set
  (MinIO, Ceph, on-prem gateways), virtual-host style on AWS.  Credentials: config
  ``access_key``/``secret_key``, else ``AWS_ACCESS_KEY_ID``/``AWS_SECRET_ACCESS_KEY``
  (+ ``AWS_SESSION_TOKEN``); region ``AWS_DEFAULT_REGION`` / ``AWS_REGION`` (default us-east-1).
* :class:`GCSStorageManager` -- the GCS JSON API (media uploads, ``alt=media`` downloads, paged
  listing); bearer token from ``GOOGLE_OAUTH_ACCESS_TOKEN`` or the GCE metadata server;
  ``STORAGE_EMULATOR_HOST`` redirects every request to an emulator (as the Google SDKs do).
* :class:`AzureStorageManager` -- Azure Blob REST with SharedKey signing (``connection_string``
  with AccountName/AccountKey, or ``account_url`` + ``credential`` = account key) or a SAS token
  ``credential``; block-blob puts, paged ``comp=list``.

Checkpoints are ``<prefix>/<storage_id>/<relative path>`` objects.  ``store_path`` /
``restore_path`` stage through a local temporary directory (``is_local = False`` tells
``core.CheckpointContext`` to upload the staged directory on exit).
"""

import base64
import contextlib
import datetime
import fnmatch
import hashlib
import hmac
import os
import pathlib
import tempfile
import urllib.parse
import xml.etree.ElementTree as ET
from typing import Any, Dict, Iterator, List, Optional, Tuple, Union

from determined_amd.storage import Selector, StorageManager, list_directory

_CHUNK = 8 << 20


def _requests():
    import requests

    return requests


class CloudStorageManager(StorageManager):
    """Shared upload / download / delete logic over four object primitives."""

    is_local = False

    def __init__(self, prefix: Optional[str] = None) -> None:
        super().__init__(tempfile.gettempdir())
        self.prefix = (prefix or "").strip("/")

    # -- object primitives (subclasses) ---------------------------------------------------------
    def _put(self, key: str, path: Optional[pathlib.Path]) -> None:  # path None: empty object
        raise NotImplementedError

    def _get(self, key: str, path: pathlib.Path) -> None:
        raise NotImplementedError

    def _list(self, prefix: str) -> Dict[str, int]:
        raise NotImplementedError

    def _delete(self, key: str) -> None:
        raise NotImplementedError

    # -- StorageManager ---------------------------------------------------------------------------
    def _key(self, storage_id: str, rel: str = "") -> str:
        parts = [p for p in (self.prefix, storage_id.strip("/"), rel) if p]
        return "/".join(parts)

    def upload(self, src: Union[str, os.PathLike], dst: str, paths: Optional[List[str]] = None) -> None:
        src = pathlib.Path(src)
        rels = sorted(list_directory(src)) if paths is None else list(paths)
        for rel in rels:
            if rel.endswith("/"):
                self._put(self._key(dst, rel), None)  # directory marker (empty directories survive)
            else:
                self._put(self._key(dst, rel), src / rel)

    def download(self, src: str, dst: Union[str, os.PathLike], selector: Selector = None) -> None:
        dst = pathlib.Path(dst)
        root = self._key(src) + "/"
        objs = self._list(root)
        if not objs:
            raise FileNotFoundError(f"checkpoint {src} not found under {self.describe()}")
        for key in sorted(objs):
            rel = key[len(root):]
            if not rel:
                continue
            if rel.endswith("/"):
                (dst / rel).mkdir(parents=True, exist_ok=True)
                continue
            if selector is not None and not selector(rel):
                continue
            (dst / rel).parent.mkdir(parents=True, exist_ok=True)
            self._get(key, dst / rel)

    def delete(self, storage_id: str, globs: Optional[List[str]] = None) -> Dict[str, int]:
        root = self._key(storage_id) + "/"
        objs = self._list(root)
        if not globs or globs == ["**/*"]:
            for key in objs:
                self._delete(key)
            return {}
        left: Dict[str, int] = {}
        for key, size in objs.items():
            rel = key[len(root):]
            if any(fnmatch.fnmatch(rel, g) or fnmatch.fnmatch(rel, g.replace("**/", "")) for g in globs) \
                    and not rel.endswith("/"):
                self._delete(key)
            else:
                left[rel] = size
        return left

    def list_files(self, storage_id: str) -> Dict[str, int]:
        root = self._key(storage_id) + "/"
        return {k[len(root):]: v for k, v in self._list(root).items() if k != root}

    @contextlib.contextmanager
    def store_path(self, dst: str) -> Iterator[pathlib.Path]:
        with tempfile.TemporaryDirectory() as td:
            yield pathlib.Path(td)
            self.upload(td, dst)

    @contextlib.contextmanager
    def restore_path(self, src: str, selector: Selector = None) -> Iterator[pathlib.Path]:
        with tempfile.TemporaryDirectory() as td:
            self.download(src, td, selector)
            yield pathlib.Path(td)

    def describe(self) -> str:
        return type(self).__name__


def _check(resp: Any, what: str) -> Any:
    if resp.status_code >= 300:
        raise RuntimeError(f"{what}: HTTP {resp.status_code}: {resp.text[:300]}")
    return resp


# ================================================================================================ S3
def _uri_encode(s: str, keep_slash: bool) -> str:
    return urllib.parse.quote(s, safe="/~" if keep_slash else "~")


def sigv4_headers(method: str, url: str, region: str, access_key: str, secret_key: str,
                  headers: Optional[Dict[str, str]] = None, payload_hash: str = "UNSIGNED-PAYLOAD",
                  now: Optional[datetime.datetime] = None, service: str = "s3",
                  session_token: Optional[str] = None) -> Dict[str, str]:
    """AWS Signature Version 4 request headers (``Authorization``, ``x-amz-date``,
    ``x-amz-content-sha256`` plus the given ones) for ``method url``."""
    now = now or datetime.datetime.now(datetime.timezone.utc)
    amz_date = now.strftime("%Y%m%dT%H%M%SZ")
    day = now.strftime("%Y%m%d")
    u = urllib.parse.urlsplit(url)
    hdrs = {k.lower(): str(v).strip() for k, v in (headers or {}).items()}
    hdrs["host"] = u.netloc
    hdrs["x-amz-date"] = amz_date
    hdrs["x-amz-content-sha256"] = payload_hash
    if session_token:
        hdrs["x-amz-security-token"] = session_token
    query = urllib.parse.parse_qsl(u.query, keep_blank_values=True)
    cq = "&".join(f"{_uri_encode(k, False)}={_uri_encode(v, False)}" for k, v in sorted(query))
    signed = ";".join(sorted(hdrs))
    canon = "\n".join([method, _uri_encode(urllib.parse.unquote(u.path) or "/", True), cq,
                       "".join(f"{k}:{hdrs[k]}\n" for k in sorted(hdrs)), signed, payload_hash])
    scope = f"{day}/{region}/{service}/aws4_request"
    to_sign = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(canon.encode()).hexdigest()])
    key = ("AWS4" + secret_key).encode()
    for part in (day, region, service, "aws4_request"):
        key = hmac.new(key, part.encode(), hashlib.sha256).digest()
    sig = hmac.new(key, to_sign.encode(), hashlib.sha256).hexdigest()
    out = {k: v for k, v in hdrs.items() if k != "host"}
    out["Authorization"] = f"AWS4-HMAC-SHA256 Credential={access_key}/{scope}, SignedHeaders={signed}, Signature={sig}"
    return out


class S3StorageManager(CloudStorageManager):
    def __init__(self, bucket: str, access_key: Optional[str] = None, secret_key: Optional[str] = None,
                 endpoint_url: Optional[str] = None, prefix: Optional[str] = None,
                 region: Optional[str] = None) -> None:
        super().__init__(prefix)
        if not bucket:
            raise ValueError("s3 checkpoint storage needs a bucket")
        self.bucket = bucket
        self.access_key = access_key or os.environ.get("AWS_ACCESS_KEY_ID", "")
        self.secret_key = secret_key or os.environ.get("AWS_SECRET_ACCESS_KEY", "")
        self.session_token = os.environ.get("AWS_SESSION_TOKEN") if not access_key else None
        if not (self.access_key and self.secret_key):
            raise ValueError("s3 checkpoint storage needs access_key/secret_key (config or AWS_* environment)")
        self.region = region or os.environ.get("AWS_DEFAULT_REGION") or os.environ.get("AWS_REGION") or "us-east-1"
        if endpoint_url:
            self.base = f"{endpoint_url.rstrip('/')}/{bucket}"
        else:
            self.base = f"https://{bucket}.s3.{self.region}.amazonaws.com"
        self.s = _requests().Session()

    @classmethod
    def from_config(cls, cfg: Dict[str, Any]) -> "S3StorageManager":
        return cls(cfg.get("bucket"), cfg.get("access_key"), cfg.get("secret_key"), cfg.get("endpoint_url"),
                   cfg.get("prefix"))

    def describe(self) -> str:
        return f"s3://{self.bucket}/{self.prefix}"

    def _req(self, method: str, key: str, query: str = "", headers: Optional[Dict[str, str]] = None, **kw: Any):
        url = f"{self.base}/{_uri_encode(key, True)}" + (f"?{query}" if query else "")
        h = sigv4_headers(method, url, self.region, self.access_key, self.secret_key, headers,
                          session_token=self.session_token)
        return self.s.request(method, url, headers=h, timeout=600, **kw)

    def _put(self, key: str, path: Optional[pathlib.Path]) -> None:
        if path is None:
            _check(self._req("PUT", key, data=b"", headers={"Content-Length": "0"}), f"s3 put {key}")
            return
        with open(path, "rb") as f:
            size = os.fstat(f.fileno()).st_size
            _check(self._req("PUT", key, data=f, headers={"Content-Length": str(size)}), f"s3 put {key}")

    def _get(self, key: str, path: pathlib.Path) -> None:
        with self._req("GET", key, stream=True) as r:
            _check(r, f"s3 get {key}")
            with open(path, "wb") as f:
                for chunk in r.iter_content(_CHUNK):
                    f.write(chunk)

    def _list(self, prefix: str) -> Dict[str, int]:
        out: Dict[str, int] = {}
        token = None
        while True:
            q = {"list-type": "2", "prefix": prefix}
            if token:
                q["continuation-token"] = token
            r = _check(self._req("GET", "", query=urllib.parse.urlencode(q)), f"s3 list {prefix}")
            root = ET.fromstring(r.content)
            ns = root.tag[: root.tag.index("}") + 1] if root.tag.startswith("{") else ""
            for c in root.findall(f"{ns}Contents"):
                out[c.findtext(f"{ns}Key")] = int(c.findtext(f"{ns}Size") or 0)
            if (root.findtext(f"{ns}IsTruncated") or "false").lower() != "true":
                return out
            token = root.findtext(f"{ns}NextContinuationToken")

    def _delete(self, key: str) -> None:
        r = self._req("DELETE", key)
        if r.status_code not in (200, 204, 404):
            _check(r, f"s3 delete {key}")


# =============================================================================================== GCS
class GCSStorageManager(CloudStorageManager):
    METADATA_TOKEN = "http://metadata.google.internal/computeMetadata/v1/instance/service-accounts/default/token"

    def __init__(self, bucket: str, prefix: Optional[str] = None) -> None:
        super().__init__(prefix)
        if not bucket:
            raise ValueError("gcs checkpoint storage needs a bucket")
        self.bucket = bucket
        emu = os.environ.get("STORAGE_EMULATOR_HOST")
        self.base = (emu if emu and "://" in emu else f"http://{emu}") if emu else "https://storage.googleapis.com"
        self.base = self.base.rstrip("/")
        self.s = _requests().Session()
        self._token: Optional[Tuple[str, float]] = None

    @classmethod
    def from_config(cls, cfg: Dict[str, Any]) -> "GCSStorageManager":
        return cls(cfg.get("bucket"), cfg.get("prefix"))

    def describe(self) -> str:
        return f"gs://{self.bucket}/{self.prefix}"

    def _auth(self) -> Dict[str, str]:
        tok = os.environ.get("GOOGLE_OAUTH_ACCESS_TOKEN")
        if tok:
            return {"Authorization": f"Bearer {tok}"}
        if os.environ.get("STORAGE_EMULATOR_HOST"):
            return {}
        import time

        if self._token is None or self._token[1] < time.time() + 60:
            r = _check(self.s.get(self.METADATA_TOKEN, headers={"Metadata-Flavor": "Google"}, timeout=10),
                       "gcs token from the metadata server")
            d = r.json()
            self._token = (d["access_token"], time.time() + float(d.get("expires_in", 300)))
        return {"Authorization": f"Bearer {self._token[0]}"}

    def _obj(self, key: str) -> str:
        return f"{self.base}/storage/v1/b/{self.bucket}/o/{urllib.parse.quote(key, safe='')}"

    def _put(self, key: str, path: Optional[pathlib.Path]) -> None:
        url = f"{self.base}/upload/storage/v1/b/{self.bucket}/o"
        params = {"uploadType": "media", "name": key}
        h = dict(self._auth(), **{"Content-Type": "application/octet-stream"})
        if path is None:
            _check(self.s.post(url, params=params, data=b"", headers=h, timeout=600), f"gcs put {key}")
            return
        with open(path, "rb") as f:
            _check(self.s.post(url, params=params, data=f, headers=h, timeout=600), f"gcs put {key}")

    def _get(self, key: str, path: pathlib.Path) -> None:
        with self.s.get(self._obj(key), params={"alt": "media"}, headers=self._auth(), stream=True, timeout=600) as r:
            _check(r, f"gcs get {key}")
            with open(path, "wb") as f:
                for chunk in r.iter_content(_CHUNK):
                    f.write(chunk)

    def _list(self, prefix: str) -> Dict[str, int]:
        out: Dict[str, int] = {}
        params = {"prefix": prefix}
        while True:
            r = _check(self.s.get(f"{self.base}/storage/v1/b/{self.bucket}/o", params=params, headers=self._auth(),
                                  timeout=60), f"gcs list {prefix}")
            d = r.json()
            for it in d.get("items", []):
                out[it["name"]] = int(it.get("size", 0))
            if not d.get("nextPageToken"):
                return out
            params = {"prefix": prefix, "pageToken": d["nextPageToken"]}

    def _delete(self, key: str) -> None:
        r = self.s.delete(self._obj(key), headers=self._auth(), timeout=60)
        if r.status_code not in (200, 204, 404):
            _check(r, f"gcs delete {key}")


# ============================================================================================= Azure
AZURE_API_VERSION = "2021-08-06"


def azure_shared_key(account: str, key_b64: str, method: str, url: str, headers: Dict[str, str]) -> str:
    """``SharedKey account:signature`` for a Blob-service request (version >= 2015-02-21 rules:
    an empty Content-Length when 0)."""
    h = {k.lower(): v for k, v in headers.items()}
    u = urllib.parse.urlsplit(url)
    clen = h.get("content-length", "")
    std = [method, h.get("content-encoding", ""), h.get("content-language", ""), "" if clen == "0" else clen,
           h.get("content-md5", ""), h.get("content-type", ""), h.get("date", ""), h.get("if-modified-since", ""),
           h.get("if-match", ""), h.get("if-none-match", ""), h.get("if-unmodified-since", ""), h.get("range", "")]
    canon_h = "".join(f"{k}:{h[k].strip()}\n" for k in sorted(h) if k.startswith("x-ms-"))
    path = u.path
    canon_r = f"/{account}{path}"
    q: Dict[str, List[str]] = {}
    for k, v in urllib.parse.parse_qsl(u.query, keep_blank_values=True):
        q.setdefault(k.lower(), []).append(v)
    for k in sorted(q):
        canon_r += f"\n{k}:{','.join(sorted(q[k]))}"
    to_sign = "\n".join(std) + "\n" + canon_h + canon_r
    sig = base64.b64encode(hmac.new(base64.b64decode(key_b64), to_sign.encode("utf-8"), hashlib.sha256).digest())
    return f"SharedKey {account}:{sig.decode()}"


class AzureStorageManager(CloudStorageManager):
    def __init__(self, container: str, connection_string: Optional[str] = None, account_url: Optional[str] = None,
                 credential: Optional[str] = None, prefix: Optional[str] = None) -> None:
        super().__init__(prefix)
        if not container:
            raise ValueError("azure checkpoint storage needs a container")
        self.container = container
        self.account = self.key = self.sas = None
        endpoint = account_url
        if connection_string:
            kv = dict(p.split("=", 1) for p in connection_string.split(";") if "=" in p)
            self.account, self.key = kv.get("AccountName"), kv.get("AccountKey")
            self.sas = kv.get("SharedAccessSignature")
            endpoint = kv.get("BlobEndpoint") or endpoint
            if not endpoint and self.account:
                proto = kv.get("DefaultEndpointsProtocol", "https")
                endpoint = f"{proto}://{self.account}.blob.{kv.get('EndpointSuffix', 'core.windows.net')}"
        elif credential:
            if "sig=" in credential:
                self.sas = credential.lstrip("?")
            else:
                self.key = credential
        if not endpoint:
            raise ValueError("azure checkpoint storage needs a connection_string or an account_url")
        self.base = endpoint.rstrip("/")
        if self.account is None:
            host = urllib.parse.urlsplit(self.base).netloc
            self.account = host.split(".")[0] if ".blob." in host else urllib.parse.urlsplit(self.base).path.strip("/")
        if not (self.key or self.sas):
            raise ValueError("azure checkpoint storage needs an account key or a SAS token")
        self.s = _requests().Session()

    @classmethod
    def from_config(cls, cfg: Dict[str, Any]) -> "AzureStorageManager":
        return cls(cfg.get("container"), cfg.get("connection_string"), cfg.get("account_url"), cfg.get("credential"),
                   cfg.get("prefix"))

    def describe(self) -> str:
        return f"azure://{self.container}/{self.prefix}"

    def _req(self, method: str, blob: str, query: str = "", headers: Optional[Dict[str, str]] = None, **kw: Any):
        path = f"/{self.container}" + (f"/{urllib.parse.quote(blob, safe='/')}" if blob else "")
        q = query
        if self.sas:
            q = f"{q}&{self.sas}" if q else self.sas
        url = f"{self.base}{path}" + (f"?{q}" if q else "")
        h = {"x-ms-version": AZURE_API_VERSION,
             "x-ms-date": datetime.datetime.now(datetime.timezone.utc).strftime("%a, %d %b %Y %H:%M:%S GMT")}
        h.update(headers or {})
        if self.key and not self.sas:
            signed_url = f"{self.base}{path}" + (f"?{query}" if query else "")
            # the canonical resource is the path of the BLOB endpoint; emulators put the account first
            h["Authorization"] = azure_shared_key(self.account, self.key, method, signed_url, h)
        return self.s.request(method, url, headers=h, timeout=600, **kw)

    def _put(self, key: str, path: Optional[pathlib.Path]) -> None:
        h = {"x-ms-blob-type": "BlockBlob", "Content-Type": "application/octet-stream"}
        if path is None:
            _check(self._req("PUT", key, headers=dict(h, **{"Content-Length": "0"}), data=b""), f"azure put {key}")
            return
        with open(path, "rb") as f:
            size = os.fstat(f.fileno()).st_size
            _check(self._req("PUT", key, headers=dict(h, **{"Content-Length": str(size)}), data=f), f"azure put {key}")

    def _get(self, key: str, path: pathlib.Path) -> None:
        with self._req("GET", key, stream=True) as r:
            _check(r, f"azure get {key}")
            with open(path, "wb") as f:
                for chunk in r.iter_content(_CHUNK):
                    f.write(chunk)

    def _list(self, prefix: str) -> Dict[str, int]:
        out: Dict[str, int] = {}
        marker = ""
        while True:
            q = {"restype": "container", "comp": "list", "prefix": prefix}
            if marker:
                q["marker"] = marker
            r = _check(self._req("GET", "", query=urllib.parse.urlencode(q)), f"azure list {prefix}")
            root = ET.fromstring(r.content)
            for b in root.iter("Blob"):
                size = b.find("Properties/Content-Length")
                out[b.findtext("Name")] = int(size.text) if size is not None and size.text else 0
            marker = root.findtext("NextMarker") or ""
            if not marker:
                return out

    def _delete(self, key: str) -> None:
        r = self._req("DELETE", key)
        if r.status_code not in (200, 202, 404):
            _check(r, f"azure delete {key}")
