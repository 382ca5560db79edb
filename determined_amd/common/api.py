"""HTTP session to the determined_amd master (reference: ``harness/determined/common/api``).

JSON over HTTP with bearer-token auth and bounded retries on connection errors.
"""

import json
import time
from typing import Any, Dict, Optional

import requests


class APIException(Exception):
    def __init__(self, status: int, message: str) -> None:
        super().__init__(f"{status}: {message}")
        self.status = status
        self.message = message


class NotFoundException(APIException):
    pass


class Session:
    def __init__(self, master_url: str, token: Optional[str] = None, max_retries: int = 5,
                 timeout: float = 60.0) -> None:
        if not master_url.startswith("http"):
            master_url = "http://" + master_url
        self.master_url = master_url.rstrip("/")
        self.token = token
        self.max_retries = max_retries
        self.timeout = timeout
        self._http = requests.Session()

    def _headers(self) -> Dict[str, str]:
        h = {"Content-Type": "application/json"}
        if self.token:
            h["Authorization"] = f"Bearer {self.token}"
        return h

    def request(self, method: str, path: str, body: Any = None, params: Optional[Dict[str, Any]] = None,
                timeout: Optional[float] = None) -> Any:
        url = self.master_url + path
        data = None if body is None else json.dumps(body, default=_json_default)
        last: Optional[Exception] = None
        for attempt in range(self.max_retries + 1):
            try:
                r = self._http.request(method, url, data=data, params=params, headers=self._headers(),
                                       timeout=timeout or self.timeout)
            except requests.ConnectionError as e:
                last = e
                time.sleep(min(2.0**attempt * 0.1, 5.0))
                continue
            if r.status_code == 404:
                raise NotFoundException(404, r.text)
            if r.status_code >= 400:
                raise APIException(r.status_code, r.text)
            if not r.content:
                return None
            return r.json()
        raise ConnectionError(f"master unreachable at {self.master_url}: {last}")

    def get(self, path: str, **kw: Any) -> Any:
        return self.request("GET", path, **kw)

    def post(self, path: str, body: Any = None, **kw: Any) -> Any:
        return self.request("POST", path, body=body, **kw)

    def delete(self, path: str, **kw: Any) -> Any:
        return self.request("DELETE", path, **kw)

    def patch(self, path: str, body: Any = None, **kw: Any) -> Any:
        return self.request("PATCH", path, body=body, **kw)


def _json_default(o: Any) -> Any:
    try:
        import numpy as np

        if isinstance(o, np.generic):
            return o.item()
        if isinstance(o, np.ndarray):
            return o.tolist()
    except ImportError:
        pass
    try:
        import torch

        if isinstance(o, torch.Tensor):
            return o.detach().cpu().tolist()
    except ImportError:
        pass
    if hasattr(o, "isoformat"):
        return o.isoformat()
    raise TypeError(f"not JSON serializable: {type(o)}")


def json_encode(o: Any) -> str:
    return json.dumps(o, default=_json_default)
