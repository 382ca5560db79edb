"""Strict experiment-config schema (expconf v0) for determined_amd: validation, defaults and merging.

The reference describes its config as JSON-Schema files with custom extensions
(``schemas/expconf/v0/*.json``: ``union``, ``optionalRef``, ``checks``, ``compareProperties``,
``eventuallyRequired``, ``disallowProperties``; Go engine ``master/pkg/schemas/extensions``) and
fills defaults / merges templates from generated Go structs.  Here the same semantics are encoded
directly as a small Python schema DSL:

* :func:`sanity_errors` -- structural validation: unknown keys are rejected at every level
  (the reference's ``"additionalProperties": false``), types, ranges, enums, patterns, unions, custom
  checks;
* :func:`completeness_errors` -- sanity plus the "eventually required" fields a config must have
  once defaults and templates have been applied;
* :func:`with_defaults` -- the reference's ``schemas.WithDefaults`` (including its runtime
  defaults and Go-side normalisations: image / environment-variable maps, ``gpu`` -> ``cuda``,
  ``--device`` strings, implicit const hyperparameters);
* :func:`merge` -- ``schemas.Merge`` (template merging: the config's own values win; unions merge
  only within the same member; bind mounts / devices append by container path).

Errors render as ``<config>.<path>: <message>``, like the reference's ``GetRenderedErrors``.
Schemas are addressed by the reference's file names (``"experiment.json"``, ``"searcher.json"``, ...);
tests/test_config_reference_cases.py replays the reference's ``schemas/test_cases/v0`` corpus.
"""

import copy
import math
import posixpath
import re
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

_MISSING = object()


def _typename(v: Any) -> str:
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "boolean"
    if isinstance(v, int):
        return "integer"
    if isinstance(v, float):
        return "number"
    if isinstance(v, str):
        return "string"
    if isinstance(v, list):
        return "array"
    if isinstance(v, dict):
        return "object"
    return type(v).__name__


def _is_type(v: Any, t: str) -> bool:
    n = _typename(v)
    if t == "number":
        return n in ("integer", "number") or (isinstance(v, float) and v.is_integer() and False)
    if t == "integer":
        return n == "integer" or (n == "number" and float(v).is_integer())
    return n == t


class Ctx:
    def __init__(self, complete: bool) -> None:
        self.complete = complete
        self.errors: List[str] = []

    def err(self, path: str, msg: str) -> None:
        self.errors.append(f"<config>{path}: {msg}")


class Node:
    """A schema node.  ``omit``: the Go struct field is ``omitempty`` (left out of marshalled
    output when unset); ``runtime``: Go fills a non-null value at runtime (e.g. a random seed)."""

    default: Any = _MISSING
    omit = False
    runtime: Any = None

    def check(self, v: Any, path: str, ctx: Ctx) -> None:
        raise NotImplementedError

    def valid(self, v: Any, complete: bool = False) -> bool:
        c = Ctx(complete)
        self.check(v, "", c)
        return not c.errors

    def defaults(self, v: Any) -> Any:
        return v

    def merge(self, a: Any, b: Any) -> Any:
        return b if a is None else a

    def emit(self, v: Any) -> Any:  # Go-marshalled form
        return v


class AnyNode(Node):
    def __init__(self, **kw: Any) -> None:
        for k, v in kw.items():
            setattr(self, k, v)

    def check(self, v, path, ctx):
        pass


class T(Node):
    """A scalar / array leaf: ``types`` is a tuple of JSON type names."""

    def __init__(self, *types: str, default: Any = _MISSING, minimum: Optional[float] = None,
                 maximum: Optional[float] = None, exclusive_minimum: Optional[float] = None, pattern: Optional[str] = None,
                 enum: Optional[Sequence[Any]] = None, const: Any = _MISSING, items: Optional[Node] = None,
                 min_items: Optional[int] = None, checks: Optional[Dict[str, Callable[[Any], bool]]] = None,
                 omit: bool = False, runtime: Any = None) -> None:
        self.types = types
        self.default = default
        self.minimum, self.maximum, self.exclusive_minimum = minimum, maximum, exclusive_minimum
        self.pattern = re.compile(pattern) if pattern else None
        self.enum = list(enum) if enum is not None else None
        self.const = const
        self.items = items
        self.min_items = min_items
        self.checks = checks or {}
        self.omit = omit
        self.runtime = runtime

    def check(self, v, path, ctx):
        if self.const is not _MISSING:
            if v != self.const or _typename(v) != _typename(self.const):
                ctx.err(path, f"value must be {self.const!r}")
            return
        if self.enum is not None:
            if v not in self.enum or (v is not None and not any(_typename(v) == _typename(e) for e in self.enum)):
                ctx.err(path, f"value must be one of {[e for e in self.enum if e is not None]}")
                return
        if self.types and not any(_is_type(v, t) for t in self.types):
            ctx.err(path, f"expected {' or '.join(self.types)}, but got {_typename(v)}")
            return
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            if self.minimum is not None and v < self.minimum:
                ctx.err(path, f"must be >= {self.minimum} but found {v}")
            if self.maximum is not None and v > self.maximum:
                ctx.err(path, f"must be <= {self.maximum} but found {v}")
            if self.exclusive_minimum is not None and v <= self.exclusive_minimum:
                ctx.err(path, f"must be > {self.exclusive_minimum} but found {v}")
        if isinstance(v, str) and self.pattern is not None and not self.pattern.search(v):
            ctx.err(path, f"does not match pattern {self.pattern.pattern!r}")
        if isinstance(v, list):
            if self.min_items is not None and len(v) < self.min_items:
                ctx.err(path, f"must have at least {self.min_items} items")
            if self.items is not None:
                for i, x in enumerate(v):
                    self.items.check(x, f"{path}[{i}]", ctx)
        if v is not None:
            for msg, ok in self.checks.items():
                if not ok(v):
                    ctx.err(path, msg)

    def defaults(self, v):
        if isinstance(v, list) and self.items is not None:
            return [self.items.defaults(x) for x in v]
        return v

    def emit(self, v):
        if isinstance(v, list) and self.items is not None:
            return [self.items.emit(x) for x in v]
        return v


class Ref(Node):
    """Reference to a named schema; ``optional`` (the ``optionalRef`` extension): null is valid too."""

    def __init__(self, name: str, optional: bool = False, default: Any = _MISSING, omit: bool = False,
                 types: Optional[Tuple[str, ...]] = None) -> None:
        self.name, self.optional, self.default, self.omit, self.types = name, optional, default, omit, types

    @property
    def target(self) -> Node:
        return SCHEMAS[self.name]

    def check(self, v, path, ctx):
        if v is None and self.optional:
            return
        if self.types is not None and not any(_is_type(v, t) for t in self.types):
            ctx.err(path, f"expected {' or '.join(t for t in self.types if t != 'null')}, but got {_typename(v)}")
            return
        self.target.check(v, path, ctx)

    def defaults(self, v):
        return self.target.defaults(v)

    def merge(self, a, b):
        if a is None:
            return b
        if b is None:
            return a
        return self.target.merge(a, b)

    def emit(self, v):
        return None if v is None else self.target.emit(v)


class Obj(Node):
    def __init__(self, props: Dict[str, Node], required: Sequence[str] = (), eventually: Sequence[str] = (),
                 additional: Any = False, checks: Optional[Dict[str, Callable[[Dict[str, Any]], bool]]] = None,
                 eventual_checks: Optional[Dict[str, Callable[[Dict[str, Any]], bool]]] = None,
                 disallow: Optional[Dict[str, str]] = None, nullable: bool = False, default: Any = _MISSING,
                 omit: bool = False, normalize: Optional[Callable[[Dict[str, Any]], Dict[str, Any]]] = None) -> None:
        self.props = props
        self.required = tuple(required)
        self.eventually = tuple(eventually)
        self.additional = additional
        self.checks = checks or {}
        self.eventual_checks = eventual_checks or {}
        self.disallow = disallow or {}
        self.nullable = nullable
        self.default = default
        self.omit = omit
        self.normalize = normalize

    def check(self, v, path, ctx):
        if v is None and self.nullable:
            return
        if not isinstance(v, dict):
            ctx.err(path, f"expected object, but got {_typename(v)}")
            return
        for k in self.required:
            if k not in v:
                ctx.err(path, f"{k} is a required property")
        if ctx.complete:
            for k in self.eventually:
                if v.get(k) is None:
                    ctx.err(path, f"{k} is a required property")
            for msg, ok in self.eventual_checks.items():
                if not ok(v):
                    ctx.err(path, msg)
        for k, x in v.items():
            sub = f"{path}.{k}"
            if k in self.disallow:
                ctx.err(sub, self.disallow[k])
                continue
            p = self.props.get(k)
            if p is not None:
                p.check(x, sub, ctx)
            elif self.additional is False:
                ctx.err(path, f"additional property {k!r} is not allowed")
            elif isinstance(self.additional, Node):
                self.additional.check(x, sub, ctx)
        for msg, ok in self.checks.items():
            if not ok(v):
                ctx.err(path, msg)

    def defaults(self, v):
        if v is None:
            return None
        v = dict(v)
        if self.normalize is not None:
            v = self.normalize(v)
        for k, p in self.props.items():
            cur = v.get(k)
            if cur is None and p.default is not _MISSING:
                cur = copy.deepcopy(p.default)
            if cur is None and p.runtime is not None:
                cur = p.runtime() if callable(p.runtime) else p.runtime
            if cur is not None:
                cur = p.defaults(cur)
            if cur is not None or k in v or not p.omit:
                v[k] = cur
        if isinstance(self.additional, Node):
            for k in list(v):
                if k not in self.props:
                    v[k] = self.additional.defaults(v[k])
        return v

    def merge(self, a, b):
        if a is None:
            return b
        if b is None or not isinstance(a, dict) or not isinstance(b, dict):
            return a
        out = dict(a)
        for k, bv in b.items():
            p = self.props.get(k, self.additional if isinstance(self.additional, Node) else None)
            av = out.get(k)
            if av is None:
                out[k] = bv
            elif p is not None:
                out[k] = p.merge(av, bv)
        return out

    def emit(self, v):
        if v is None:
            return None
        out = {}
        for k, p in self.props.items():
            if k in v:
                if v[k] is None and p.omit:
                    continue
                out[k] = p.emit(v[k])
            elif not p.omit:
                out[k] = None
        for k, x in v.items():
            if k not in self.props:
                out[k] = self.additional.emit(x) if isinstance(self.additional, Node) else x
        return out


class Union(Node):
    """The ``union`` extension: valid iff exactly one member validates; otherwise the error of the
    first member whose key selects the value, under the default message."""

    def __init__(self, items: Sequence[Tuple[str, Node]], message: str = "union failed to validate",
                 default: Any = _MISSING, omit: bool = False, pre: Optional[Callable[[Any], Any]] = None,
                 common: Sequence[str] = ()) -> None:
        self.items = list(items)
        self.common = tuple(common)  # fields shared by every member (Go: fields outside the union pointers)
        self.message = message
        self.default = default
        self.omit = omit
        self.pre = pre  # Go-side normalisation before defaults

    @staticmethod
    def selects(key: str, v: Any) -> bool:
        if key == "always":
            return True
        if key == "never":
            return False
        if key.startswith("not:"):
            return not Union.selects(key[4:], v)
        if key.startswith("const:"):
            name, _, val = key[6:].partition("=")
            return isinstance(v, dict) and isinstance(v.get(name), str) and v.get(name) == val
        if key.startswith("singleproperty:"):
            return isinstance(v, dict) and len(v) == 1 and key[15:] in v
        if key.startswith("type:"):
            return _typename(v) == key[5:]
        if key.startswith("hasattr:"):
            return isinstance(v, dict) and key[8:] in v
        raise ValueError(f"bad union key {key!r}")

    def member(self, v: Any) -> Optional[Node]:
        for key, node in self.items:
            if node.valid(v):
                return node
        for key, node in self.items:
            if self.selects(key, v):
                return node
        return None

    def check(self, v, path, ctx):
        valid, selected = [], None
        for key, node in self.items:
            c = Ctx(ctx.complete)
            node.check(v, path, c)
            if c.errors:
                if selected is None and self.selects(key, v):
                    selected = c.errors
            else:
                valid.append(node)
        if len(valid) == 1:
            return
        if len(valid) > 1:
            ctx.err(path, "bug in validation! multiple union members matched")
            return
        ctx.err(path, self.message)
        if selected:
            ctx.errors.extend(selected)

    def defaults(self, v):
        if self.pre is not None:
            v = self.pre(v)
        m = self.member(v)
        return m.defaults(v) if m is not None else v

    def merge(self, a, b):
        if a is None:
            return b
        if b is None:
            return a
        ma, mb = self.member(a), self.member(b)
        if ma is not None and ma is mb:
            return ma.merge(a, b)
        if isinstance(a, dict) and isinstance(b, dict):
            a = dict(a)  # a different (or no) member in the template: only the shared fields carry over
            for k in self.common:
                if a.get(k) is None and b.get(k) is not None:
                    a[k] = b[k]
        return a

    def emit(self, v):
        m = self.member(v)
        return m.emit(v) if m is not None else v


class AllOf(Node):
    def __init__(self, *nodes: Node) -> None:
        self.nodes = nodes

    def check(self, v, path, ctx):
        for n in self.nodes:
            n.check(v, path, ctx)

    def defaults(self, v):
        return self.nodes[0].defaults(v)

    def merge(self, a, b):
        return self.nodes[0].merge(a, b)

    def emit(self, v):
        return self.nodes[0].emit(v)


# ----------------------------------------------------------------------------------------------- helpers
def _opt(*types: str) -> Tuple[str, ...]:
    return tuple(types) + ("null",)


def S(default: Any = None, **kw: Any) -> T:
    return T("string", "null", default=default, **kw)


def I(default: Any = None, **kw: Any) -> T:  # noqa: E743
    return T("integer", "null", default=default, **kw)


def N(default: Any = None, **kw: Any) -> T:
    return T("number", "null", default=default, **kw)


def B(default: Any = None, **kw: Any) -> T:
    return T("boolean", "null", default=default, **kw)


def StrList(default: Any = (), **kw: Any) -> T:
    return T("array", "null", default=list(default) if default is not None else None, items=T("string"), **kw)


def _no_dotdot(p: str) -> bool:
    return not (p == ".." or p.startswith("../") or p.endswith("/..") or "/../" in p)


def _subdir(o: Dict[str, Any]) -> bool:
    sp, hp = o.get("storage_path"), o.get("host_path")
    if sp is None:
        return True
    norm = posixpath.normpath(sp)
    if not sp.startswith("/"):
        return not (norm == ".." or norm.startswith("../"))
    if hp is None:
        return True
    hpn = posixpath.normpath(hp)
    return norm == hpn or norm.startswith(hpn.rstrip("/") + "/")


def _cmp(a: str, b: str, op: str, msg: str) -> Dict[str, Callable[[Dict[str, Any]], bool]]:
    def ok(o: Dict[str, Any]) -> bool:
        x, y = o.get(a), o.get(b)
        if not isinstance(x, (int, float)) or not isinstance(y, (int, float)):
            return True
        return x < y if op == "<" else x <= y
    return {msg: ok}


_SAVE = {"save_experiment_best": I(0, minimum=0), "save_trial_best": I(1, minimum=0),
         "save_trial_latest": I(1, minimum=0)}


def _storage(kind: str, props: Dict[str, Node], eventually: Sequence[str] = (),
             checks: Optional[Dict[str, Callable]] = None, eventual_checks: Optional[Dict[str, Callable]] = None) -> Obj:
    return Obj({"type": T(const=kind), **props, **_SAVE}, required=("type",), eventually=eventually, checks=checks,
               eventual_checks=eventual_checks)


_PREFIX = S(None, checks={"prefix cannot contain /../": _no_dotdot})


def _length_member(unit: str) -> Obj:
    return Obj({unit: T("integer", minimum=0)}, required=(unit,))


def _pos_length_member(unit: str) -> Obj:
    return Obj({unit: T("integer", minimum=1)}, required=(unit,))


_LEN_MSG = 'a length object must have one attribute named "batches", "records", or "epochs"'


# ----- Go-side normalisations applied with defaults
def _image_pre(v: Any) -> Any:
    if isinstance(v, str):
        return {"cpu": v, "cuda": v, "rocm": v}
    if isinstance(v, dict):
        v = dict(v)
        if v.get("gpu") is not None and v.get("cuda") is None:
            v["cuda"] = v["gpu"]
        v.pop("gpu", None)
    return v


def _envvars_pre(v: Any) -> Any:
    if isinstance(v, list):
        return {"cpu": list(v), "cuda": list(v), "rocm": list(v)}
    if isinstance(v, dict):
        v = dict(v)
        if v.get("gpu") is not None and v.get("cuda") is None:
            v["cuda"] = v["gpu"]
        v.pop("gpu", None)
    return v


def _device_pre(v: Any) -> Any:
    if isinstance(v, str):
        parts = v.split(":")
        d = {"host_path": parts[0], "container_path": parts[1] if len(parts) > 1 else parts[0]}
        if len(parts) > 2:
            d["mode"] = parts[2]
        return d
    return v


def _hp_pre(v: Any) -> Any:
    if isinstance(v, dict) and "type" in v:
        return v
    if isinstance(v, dict) and v:
        return v  # nested
    return {"type": "const", "val": v}


_DEFAULT_IMAGE = "determinedai/pytorch-rocm:mi355x"


def _random_seed() -> int:
    import random

    return random.randrange(2**31)


class _Hparam(Union):
    """hyperparameter.json: typed members, nested dicts, implicit consts; merges nested dicts recursively."""

    def defaults(self, v):
        v = _hp_pre(v)
        if isinstance(v, dict) and "type" not in v:
            return {k: self.defaults(x) for k, x in v.items()}
        m = self.member(v)
        return m.defaults(v) if m is not None else v

    def merge(self, a, b):
        a, b = _hp_pre(a), _hp_pre(b)
        if isinstance(a, dict) and "type" not in a and isinstance(b, dict) and "type" not in b:
            out = {k: self.defaults(x) for k, x in a.items()}
            for k, x in b.items():
                out[k] = self.merge(out[k], x) if k in out else self.defaults(x)
            return out
        return a

    def emit(self, v):
        v = _hp_pre(v)
        if isinstance(v, dict) and "type" not in v:
            return {k: self.emit(x) for k, x in v.items()}
        m = self.member(v)
        return m.emit(v) if m is not None else v


class _AppendByContainerPath(T):
    """bind mounts / devices: merged lists append the template's entries whose container_path is new."""

    def merge(self, a, b):
        if a is None:
            return b
        if b is None:
            return a
        a = [_device_pre(x) for x in a]
        seen = {x.get("container_path") for x in a if isinstance(x, dict)}
        return a + [x for x in (_device_pre(y) for y in b) if isinstance(x, dict) and x.get("container_path") not in seen]


def _pod_spec_check(spec: Dict[str, Any]) -> List[Tuple[str, str]]:
    out = []
    for i, c in enumerate(((spec.get("spec") or {}).get("containers") or [])):
        if isinstance(c, dict) and c.get("name") == "determined-container":
            out.append((f".spec.containers[{i}]", "container name determined-container is not configurable"))
    return out


class _PodSpec(Node):
    omit = False
    default = None

    def check(self, v, path, ctx):
        if v is None:
            return
        if not isinstance(v, dict):
            ctx.err(path, f"expected object, but got {_typename(v)}")
            return
        for k, msg in (("name", "pod Name is not a configurable option"),
                       ("name_space", "pod NameSpace is not a configurable option")):
            if k in v:
                ctx.err(f"{path}.{k}", msg)
        for sub, msg in _pod_spec_check(v):
            ctx.err(path + sub, msg)

    def defaults(self, v):
        return v


def _grid_check(v: Any, path: str, ctx: Ctx) -> None:
    """check-grid-hyperparameter.json: every int / double / log hyperparameter needs a count."""
    if isinstance(v, list):
        for i, x in enumerate(v):
            _grid_check(x, f"{path}[{i}]", ctx)
    elif isinstance(v, dict) and "type" not in v:
        for k, x in v.items():
            _grid_check(x, f"{path}.{k}", ctx)
    elif isinstance(v, dict) and v.get("type") in ("double", "log", "int") and v.get("count") is None:
        ctx.err(path, "grid search is in use but count was not provided")


class _GridCheck(Node):
    def check(self, v, path, ctx):
        _grid_check(v, path, ctx)


class _Experiment(Obj):
    def check(self, v, path, ctx):
        super().check(v, path, ctx)
        if isinstance(v, dict) and isinstance(v.get("searcher"), dict) and v["searcher"].get("name") == "grid":
            _grid_check(v.get("hyperparameters") or {}, f"{path}.hyperparameters", ctx)


# ----------------------------------------------------------------------------------------------- schemas
SCHEMAS: Dict[str, Node] = {}

_MODES = (None, "aggressive", "standard", "conservative")
_SRCH_COMMON = {"metric": S(None), "smaller_is_better": B(True), "source_trial_id": I(None),
                "source_checkpoint_uuid": S(None)}


def _searcher(name: str, props: Dict[str, Node], eventually: Sequence[str], additional: Any = False) -> Obj:
    return Obj({"name": T(const=name), **props, **_SRCH_COMMON}, required=("name",), eventually=eventually,
               additional=additional)


SCHEMAS.update({
    "azure.json": _storage("azure", {"container": S(None), "connection_string": S(None),
                                     "account_url": S(None, omit=True), "credential": S(None, omit=True)},
                           eventually=("container",),
                           checks={"credential and connection_string must not both be set":
                                   lambda o: not (o.get("credential") is not None and o.get("connection_string") is not None)},
                           eventual_checks={"Exactly one of connection_string or account_url must be set":
                                            lambda o: (o.get("connection_string") is None) != (o.get("account_url") is None)}),
    "shared-fs.json": _storage("shared_fs", {"host_path": S(None), "storage_path": S(None), "propagation": S("rprivate"),
                                             "container_path": S(None, omit=True), "checkpoint_path": S(None, omit=True),
                                             "tensorboard_path": S(None, omit=True)},
                               eventually=("host_path",),
                               checks={"storage_path must either be a relative directory or a subdirectory of host_path":
                                       _subdir}),
    "directory.json": _storage("directory", {"container_path": S(None)}, eventually=("container_path",)),
    "s3.json": _storage("s3", {"access_key": S(None), "bucket": S(None), "secret_key": S(None), "endpoint_url": S(None),
                               "prefix": _PREFIX}, eventually=("bucket",)),
    "gcs.json": _storage("gcs", {"bucket": S(None), "prefix": _PREFIX}, eventually=("bucket",)),
    "bind-mount.json": Obj({"host_path": T("string", checks={"host_path must be an absolute path": lambda p: p.startswith("/")}),
                            "container_path": T("string", checks={'container_path must not be "."': lambda p: p != "."}),
                            "read_only": B(False), "propagation": S("rprivate")},
                           required=("host_path", "container_path")),
    "device.json": Obj({"host_path": T("string"), "container_path": T("string"), "mode": S("mrw")},
                       required=("host_path", "container_path")),
    "length.json": Union([(f"singleproperty:{u}", _length_member(u)) for u in ("batches", "records", "epochs")], _LEN_MSG),
    "check-positive-length.json": Union([(f"singleproperty:{u}", _pos_length_member(u))
                                         for u in ("batches", "records", "epochs")], _LEN_MSG),
    "hyperparameter-int.json": Obj({"type": T(const="int"), "minval": T("integer"), "maxval": T("integer"),
                                    "count": I(None, minimum=1, omit=True)},
                                   required=("type", "minval", "maxval"),
                                   checks=_cmp("minval", "maxval", "<", "minval must be less than maxval")),
    "hyperparameter-double.json": Obj({"type": T(const="double"), "minval": T("number"), "maxval": T("number"),
                                       "count": I(None, minimum=1, omit=True)},
                                      required=("type", "minval", "maxval"),
                                      checks=_cmp("minval", "maxval", "<", "minval must be less than maxval")),
    "hyperparameter-log.json": Obj({"type": T(const="log"), "minval": T("number"), "maxval": T("number"),
                                    "base": T("number", exclusive_minimum=0), "count": I(None, minimum=1, omit=True)},
                                   required=("type", "minval", "maxval", "base"),
                                   checks=_cmp("minval", "maxval", "<", "minval must be less than maxval")),
    "hyperparameter-const.json": Obj({"type": T(const="const"), "val": AnyNode()}, required=("type", "val")),
    "hyperparameter-categorical.json": Obj({"type": T(const="categorical"), "vals": T("array", min_items=1)},
                                           required=("type", "vals")),
    "kerberos.json": Obj({"config_file": T("string")}, required=("config_file",)),
    "security.json": Obj({"kerberos": Ref("kerberos.json", optional=True, default=None)}),
    "log-action-cancel-retries.json": Obj({"type": T(const="cancel_retries")}, required=("type",)),
    "log-action-exclude-node.json": Obj({"type": T(const="exclude_node")}, required=("type",)),
    "log-policy.json": Obj({"pattern": T("string"), "action": Ref("log-action.json")}, required=("pattern", "action")),
    "optimizations.json": Obj({
        "aggregation_frequency": I(1, minimum=1), "auto_tune_tensor_fusion": B(False),
        "average_aggregated_gradients": B(True), "average_training_metrics": B(True),
        "gradient_compression": B(False), "grad_updates_size_file": S(None),
        "mixed_precision": T(enum=(None, "O0", "O1", "O2", "O3"), default="O0"),
        "tensor_fusion_cycle_time": I(1, minimum=0), "tensor_fusion_threshold": I(64, minimum=0)}),
    "profiling.json": Obj({"enabled": B(False), "begin_on_batch": I(0, minimum=0), "end_after_batch": I(None, minimum=0),
                           "sync_timings": B(True)},
                          checks=_cmp("begin_on_batch", "end_after_batch", "<=",
                                      "begin_on_batch must be less than end_after_batch")),
    "proxy-port.json": Obj({"proxy_port": T("number"), "proxy_tcp": B(False), "unauthenticated": B(False),
                            "default_service_id": B(False)}, required=("proxy_port",)),
    "registry-auth.json": Obj({k: S(None, omit=True) for k in ("username", "password", "auth", "email", "serveraddress",
                                                               "identitytoken", "registrytoken")}),
    "reproducibility.json": Obj({"experiment_seed": I(None, minimum=0, runtime=_random_seed)},
                                eventually=("experiment_seed",)),
    "retention-policy.json": Obj({"log_retention_days": I(None, minimum=-1, maximum=32767)},
                                 eventually=("log_retention_days",)),
    "hpc-cluster-pbs.json": Obj({"slots_per_node": I(None, minimum=1, omit=True),
                                 "pbsbatch_args": StrList(None, omit=True)}),
    "hpc-cluster-slurm.json": Obj({"slots_per_node": I(None, minimum=1, omit=True), "gpu_type": S(None, omit=True),
                                   "sbatch_args": StrList(None, omit=True)}),
    "environment-image-map.json": Obj({"cpu": S(None, runtime=_DEFAULT_IMAGE), "cuda": S(None, runtime=_DEFAULT_IMAGE),
                                       "rocm": S(None, runtime=_DEFAULT_IMAGE), "gpu": S(None, omit=True)},
                                      eventually=("cpu", "cuda", "rocm")),
    "environment-variables-map.json": Obj({"cpu": StrList([]), "cuda": StrList([]), "rocm": StrList([]),
                                           "gpu": StrList(None, omit=True)}),
    "test-sub.json": Obj({"val_y": S("default_y")}),
    "test-union-a.json": Obj({"type": T(const="a"), "val_a": T("integer"), "common_val": S("default-common-val")},
                             required=("type", "val_a")),
    "test-union-b.json": Obj({"type": T(const="b"), "val_b": T("integer"), "common_val": S("default-common-val")},
                             required=("type", "val_b")),
})

SCHEMAS["environment-image.json"] = Union([("never", Ref("environment-image-map.json")), ("never", T("string"))],
                                          "is neither a string nor a map of cpu, cuda, or rocm to strings", pre=_image_pre)
SCHEMAS["environment-variables.json"] = Union(
    [("never", Ref("environment-variables-map.json")), ("never", T("array", items=T("string")))],
    "is neither a list of strings nor a map of cpu, cuda, or rocm to lists of strings", pre=_envvars_pre)
SCHEMAS["proxy-ports.json"] = T("array", items=Ref("proxy-port.json"))
SCHEMAS["bind-mounts.json"] = _AppendByContainerPath("array", items=Ref("bind-mount.json"))
SCHEMAS["devices.json"] = _AppendByContainerPath("array", items=Union(
    [("never", Ref("device.json")), ("never", T("string", pattern=r"^/[^:]*:/[^:]*(:[rwm]*)?"))],
    "is neither a list of --device strings nor a map containing host_path, container_path, and mode", pre=_device_pre))
SCHEMAS["searcher-length.json"] = Union([("not:type:object", T("integer", minimum=0)),
                                         ("always", Ref("check-positive-length.json"))])
SCHEMAS["hyperparameter.json"] = _Hparam([
    ("const:type=int", Ref("hyperparameter-int.json")), ("const:type=double", Ref("hyperparameter-double.json")),
    ("const:type=log", Ref("hyperparameter-log.json")), ("const:type=const", Ref("hyperparameter-const.json")),
    ("const:type=categorical", Ref("hyperparameter-categorical.json")),
    ("always", Obj({}, additional=Ref("hyperparameter.json"), checks={
        "if a hyperparameter object's [\"type\"] is set, it must be one of \"int\", \"double\", \"log\", const\", or "
        "\"categorical\"": lambda o: "type" not in o})),
    ("never", T("string", "integer", "number", "boolean", "array", "null")),
])
SCHEMAS["hyperparameters.json"] = Obj({}, additional=Ref("hyperparameter.json"))
SCHEMAS["check-grid-hyperparameter.json"] = _GridCheck()
SCHEMAS["log-action.json"] = Union([("const:type=cancel_retries", Ref("log-action-cancel-retries.json")),
                                    ("const:type=exclude_node", Ref("log-action-exclude-node.json"))],
                                   "is not an object where object[\"type\"] is one of 'cancel_retries' or 'exclude_node'")
SCHEMAS["checkpoint-storage.json"] = Union(
    [(f"const:type={k}", Ref(f"{f}.json")) for k, f in (("shared_fs", "shared-fs"), ("directory", "directory"), ("s3", "s3"),
                                                       ("gcs", "gcs"), ("azure", "azure"))],
    "is not an object where object[\"type\"] is one of 'shared_fs', 'directory', 's3', 'gcs', or 'azure'",
    common=tuple(_SAVE))
SCHEMAS["tensorboard-storage.json"] = Union(
    [(f"const:type={k}", Obj({kk: vv for kk, vv in SCHEMAS[f"{f}.json"].props.items() if kk not in _SAVE},  # type: ignore
                             required=("type",), disallow={s: "this field is deprecated and will be ignored" for s in _SAVE}))
     for k, f in (("shared_fs", "shared-fs"), ("s3", "s3"), ("gcs", "gcs"))],
    "this field is deprecated and will be ignored")
_SLEN = Ref("searcher-length.json", optional=True, default=None, types=("object", "integer", "null"))
_PLEN = Ref("check-positive-length.json", optional=True, default=None, types=("object", "null"))
SCHEMAS.update({
    "searcher-single.json": _searcher("single", {"max_length": _SLEN}, ("max_length", "metric")),
    "searcher-random.json": _searcher("random", {"max_concurrent_trials": I(16, minimum=0),
                                                 "max_trials": I(None, minimum=1), "max_length": _SLEN},
                                      ("max_trials", "max_length", "metric")),
    "searcher-grid.json": _searcher("grid", {"max_concurrent_trials": I(16, minimum=0), "max_length": _SLEN},
                                    ("max_length", "metric")),
    "searcher-async-halving.json": _searcher("async_halving", {
        "num_rungs": I(None, minimum=1), "max_length": _PLEN, "max_trials": I(None, minimum=1),
        "divisor": N(4, exclusive_minimum=1), "max_concurrent_trials": I(16, minimum=0), "stop_once": B(False)},
        ("num_rungs", "max_length", "max_trials", "metric")),
    "searcher-adaptive-asha.json": _searcher("adaptive_asha", {
        "bracket_rungs": T("array", "null", default=[], items=T("integer")), "max_trials": I(None, minimum=1),
        "mode": T(enum=_MODES, default="standard"), "divisor": N(4, exclusive_minimum=1),
        "max_rungs": I(5, minimum=1), "max_concurrent_trials": I(16, minimum=0), "max_length": _SLEN,
        "stop_once": B(False)}, ("max_length", "max_trials", "metric")),
    "searcher-custom.json": _searcher("custom", {"unit": T(enum=("batches", "records", "epochs", None), default=None)},
                                      ("metric",), additional=True),
    "searcher-sync-halving.json": _searcher("sync_halving", {
        "budget": _PLEN, "num_rungs": I(None, minimum=1), "max_length": _PLEN, "divisor": N(4, exclusive_minimum=1),
        "train_stragglers": B(True)}, ("num_rungs", "max_length", "budget", "metric")),
    "searcher-adaptive.json": _searcher("adaptive", {
        "budget": Ref("length.json", optional=True, default=None), "bracket_rungs": T("array", "null", default=[],
                                                                                        items=T("integer")),
        "mode": T(enum=_MODES, default="standard"), "divisor": N(4, exclusive_minimum=1),
        "max_rungs": I(5, minimum=1), "max_length": _PLEN, "train_stragglers": B(True)},
        ("budget", "max_length", "metric")),
    "searcher-adaptive-simple.json": _searcher("adaptive_simple", {
        "max_trials": I(None, minimum=1, maximum=2000), "mode": T(enum=_MODES, default="standard"),
        "divisor": N(4, exclusive_minimum=1), "max_rungs": I(5, minimum=1), "max_length": _PLEN},
        ("max_trials", "max_length", "metric")),
})
_SEARCHERS = ("single", "random", "grid", "async_halving", "adaptive_asha", "custom", "sync_halving", "adaptive",
              "adaptive_simple")
SCHEMAS["searcher.json"] = Union(
    [(f"const:name={k}", Ref(f"searcher-{k.replace('_', '-')}.json")) for k in _SEARCHERS],
    "is not an object where object[\"name\"] is one of 'single', 'random', 'grid', 'custom', or 'adaptive_asha'",
    common=tuple(_SRCH_COMMON))
SCHEMAS["resources.json"] = Obj({
    "agent_label": S(None, omit=True), "devices": Ref("devices.json", optional=True, default=[]),
    "is_single_node": B(None), "max_slots": I(None), "native_parallel": B(False),
    "priority": I(None, minimum=1, maximum=99), "resource_pool": S(""),
    "shm_size": T("integer", "string", "null", default=None,
                  checks={"must be a valid memory size": lambda v: not isinstance(v, str) or bool(
                      re.match(r"^([0-9]*[.])?[0-9]+ ?(([kmgtpKMGTP]([iI]?[bB])?)|([bB]))?$", v))}),
    "slots": I(None, omit=True), "slots_per_trial": I(1, minimum=0), "weight": N(1)})
SCHEMAS["environment.json"] = Obj({
    "image": Ref("environment-image.json", optional=True, default={}, types=("object", "string", "null")),
    "environment_variables": Ref("environment-variables.json", optional=True, default=[],
                                 types=("object", "array", "null")),
    "proxy_ports": Ref("proxy-ports.json", optional=True, default=[]),
    "ports": T("object", "null", default={}, checks={"port values must be integers": lambda o: all(
        isinstance(x, int) and not isinstance(x, bool) for x in o.values())}),
    "force_pull_image": B(False), "registry_auth": Ref("registry-auth.json", optional=True, default=None),
    "add_capabilities": StrList([]), "drop_capabilities": StrList([]), "pod_spec": _PodSpec()},
    eventually=("image",))
SCHEMAS["test-union.json"] = Union([("const:type=a", Ref("test-union-a.json")), ("const:type=b", Ref("test-union-b.json"))],
                                   "bad test union")
SCHEMAS["test-root.json"] = Obj({
    "val_x": T("integer"), "sub_obj": Ref("test-sub.json", optional=True, default={}),
    "sub_union": Ref("test-union.json", optional=True, default=None),
    "runtime_defaultable": I(None, runtime=42), "defaulted_array": StrList([]), "nodefault_array": StrList(None)},
    required=("val_x",))
SCHEMAS["experiment.json"] = _Experiment({
    "bind_mounts": Ref("bind-mounts.json", optional=True, default=[]),
    "checkpoint_policy": T(enum=(None, "best", "all", "none"), default="best"),
    "checkpoint_storage": Ref("checkpoint-storage.json", optional=True, default=None),
    "data": T("object", "null", default={}),
    "data_layer": T("object", "null", default=None, omit=True),
    "debug": B(False), "description": S(None),
    "entrypoint": T("string", "array", "null", default=None, items=T("string")),
    "environment": Ref("environment.json", optional=True, default={}),
    "hyperparameters": Ref("hyperparameters.json", optional=True, default={}),
    "internal": T("null", default=None, omit=True),
    "labels": StrList([]),
    "log_policies": T("array", "null", default=[], items=Ref("log-policy.json")),
    "retention_policy": Ref("retention-policy.json", optional=True, default=None, omit=True),
    "max_restarts": I(5, minimum=0),
    "min_checkpoint_period": Ref("length.json", optional=True, default={"batches": 0}),
    "min_validation_period": Ref("length.json", optional=True, default={"batches": 0}),
    "name": S(None, runtime=lambda: "Experiment (unnamed)"),
    "optimizations": Ref("optimizations.json", optional=True, default={}),
    "pbs": Ref("hpc-cluster-pbs.json", optional=True, default={}),
    "perform_initial_validation": B(False),
    "profiling": Ref("profiling.json", optional=True, default={}),
    "project": S(""), "records_per_epoch": I(0),
    "reproducibility": Ref("reproducibility.json", optional=True, default={}),
    "resources": Ref("resources.json", optional=True, default={}),
    "scheduling_unit": I(100, minimum=1),
    "searcher": Ref("searcher.json", optional=True, default=None),
    "security": Ref("security.json", optional=True, default=None, omit=True),
    "slurm": Ref("hpc-cluster-slurm.json", optional=True, default={}),
    "tensorboard_storage": Ref("tensorboard-storage.json", optional=True, default=None, omit=True),
    "workspace": S(""),
}, eventually=("checkpoint_storage", "name", "hyperparameters", "reproducibility", "searcher"))


# ----------------------------------------------------------------------------------------------- API
def _schema(name: str) -> Node:
    name = name.rsplit("/", 1)[-1]
    if name not in SCHEMAS:
        raise KeyError(f"no schema named {name!r}")
    return SCHEMAS[name]


def sanity_errors(value: Any, name: str = "experiment.json") -> List[str]:
    """Structural errors of ``value`` against the named schema (unknown keys included)."""
    ctx = Ctx(False)
    _schema(name).check(value, "", ctx)
    return ctx.errors


def completeness_errors(value: Any, name: str = "experiment.json") -> List[str]:
    """Sanity errors plus missing 'eventually required' fields (a config ready to run)."""
    ctx = Ctx(True)
    _schema(name).check(value, "", ctx)
    return ctx.errors


def with_defaults(value: Any, name: str = "experiment.json") -> Any:
    """``value`` with every unset field filled (Go-marshalled form: normalised unions, nulls kept)."""
    node = _schema(name)
    return node.emit(node.defaults(copy.deepcopy(value)))


def merge(value: Any, template: Any, name: str = "experiment.json") -> Any:
    """``value`` merged over ``template`` (the value's own settings win)."""
    node = _schema(name)
    return node.emit(node.merge(copy.deepcopy(value), copy.deepcopy(template)))


def is_integer(v: Any) -> bool:
    return isinstance(v, int) and not isinstance(v, bool) or (isinstance(v, float) and math.isfinite(v) and v.is_integer())
