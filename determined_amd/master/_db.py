"""Master persistence (reference: ``master/internal/db`` on Postgres; here sqlite in WAL mode).

All JSON-shaped columns are stored as TEXT.  The master holds one connection guarded by its
global lock; sqlite is more than enough for one node's experiments, trials and metrics.
"""

import json
import sqlite3
import threading
import time
from typing import Any, Dict, Iterable, List, Optional

SCHEMA = """
CREATE TABLE IF NOT EXISTS experiments (
  id INTEGER PRIMARY KEY AUTOINCREMENT, name TEXT, state TEXT, config TEXT, model_def BLOB,
  parent_id INTEGER, archived INTEGER DEFAULT 0, progress REAL DEFAULT 0, start_time REAL, end_time REAL,
  notes TEXT DEFAULT '', searcher_snapshot TEXT, owner TEXT DEFAULT 'determined', project TEXT DEFAULT 'Uncategorized',
  workspace TEXT DEFAULT 'Uncategorized', description TEXT DEFAULT '', labels TEXT DEFAULT '[]', unmanaged INTEGER DEFAULT 0);
CREATE TABLE IF NOT EXISTS trials (
  id INTEGER PRIMARY KEY AUTOINCREMENT, experiment_id INTEGER, request_id INTEGER, state TEXT, hparams TEXT,
  seed INTEGER, restarts INTEGER DEFAULT 0, run_id INTEGER DEFAULT 0, start_time REAL, end_time REAL,
  latest_checkpoint TEXT, total_batches INTEGER DEFAULT 0, searcher_metric REAL, best_validation REAL,
  runner_state TEXT DEFAULT '', searcher_state TEXT DEFAULT '{}', warm_start_checkpoint TEXT);
CREATE INDEX IF NOT EXISTS trials_exp ON trials(experiment_id);
CREATE TABLE IF NOT EXISTS metrics (
  id INTEGER PRIMARY KEY AUTOINCREMENT, trial_id INTEGER, trial_run_id INTEGER, group_name TEXT,
  steps_completed INTEGER, metrics TEXT, batch_metrics TEXT, ts REAL);
CREATE INDEX IF NOT EXISTS metrics_trial ON metrics(trial_id, group_name);
CREATE TABLE IF NOT EXISTS checkpoints (
  uuid TEXT PRIMARY KEY, trial_id INTEGER, experiment_id INTEGER, task_id TEXT, allocation_id TEXT,
  state TEXT, resources TEXT, metadata TEXT, steps_completed INTEGER, report_time REAL, searcher_metric REAL);
CREATE INDEX IF NOT EXISTS ckpt_trial ON checkpoints(trial_id);
CREATE TABLE IF NOT EXISTS task_logs (
  id INTEGER PRIMARY KEY AUTOINCREMENT, task_id TEXT, allocation_id TEXT, rank INTEGER, ts REAL, log TEXT);
CREATE INDEX IF NOT EXISTS logs_task ON task_logs(task_id, id);
CREATE TABLE IF NOT EXISTS models (
  id INTEGER PRIMARY KEY AUTOINCREMENT, name TEXT UNIQUE, description TEXT DEFAULT '', metadata TEXT DEFAULT '{}',
  labels TEXT DEFAULT '[]', creation_time REAL, archived INTEGER DEFAULT 0, notes TEXT DEFAULT '');
CREATE TABLE IF NOT EXISTS model_versions (
  id INTEGER PRIMARY KEY AUTOINCREMENT, model_id INTEGER, version INTEGER, checkpoint_uuid TEXT, name TEXT,
  comment TEXT DEFAULT '', metadata TEXT DEFAULT '{}', creation_time REAL);
CREATE TABLE IF NOT EXISTS tasks (
  id TEXT PRIMARY KEY, type TEXT, state TEXT, config TEXT, start_time REAL, end_time REAL, exit_code INTEGER);
CREATE TABLE IF NOT EXISTS webhooks (
  id INTEGER PRIMARY KEY AUTOINCREMENT, url TEXT, triggers TEXT, webhook_type TEXT DEFAULT 'DEFAULT');
CREATE TABLE IF NOT EXISTS templates (name TEXT PRIMARY KEY, config TEXT);
CREATE TABLE IF NOT EXISTS allocation_history (
  alloc_id TEXT PRIMARY KEY, task_id TEXT, kind TEXT, experiment_id INTEGER, owner TEXT, resource_pool TEXT,
  slots INTEGER, start_time REAL, end_time REAL);
CREATE TABLE IF NOT EXISTS pool_bindings (pool TEXT, workspace_id INTEGER, PRIMARY KEY (pool, workspace_id));
CREATE TABLE IF NOT EXISTS trial_source_infos (
  trial_id INTEGER, checkpoint_uuid TEXT, source_type TEXT, model_id INTEGER, model_version INTEGER,
  PRIMARY KEY (trial_id, checkpoint_uuid, source_type));
"""

MIGRATIONS = [("experiments", "external_id", "TEXT"), ("trials", "external_id", "TEXT"), ("tasks", "proxy", "TEXT"),
              ("models", "workspace", "TEXT DEFAULT 'Uncategorized'"), ("trials", "log_retention_days", "INTEGER")]

# tables whose writes feed the master's event stream (GET /api/v1/stream, the web UI)
STREAMED = {"experiments": "experiment", "trials": "trial", "checkpoints": "checkpoint", "tasks": "task",
            "models": "model", "model_versions": "model_version", "metrics": "metrics"}

JSON_COLS = {"config", "hparams", "metrics", "batch_metrics", "resources", "metadata", "searcher_snapshot", "labels",
             "searcher_state", "triggers", "proxy"}


class DB:
    def __init__(self, path: str = ":memory:") -> None:
        self.path = path
        self.conn = sqlite3.connect(path, check_same_thread=False, isolation_level=None)
        self.conn.row_factory = sqlite3.Row
        if path != ":memory:":
            self.conn.execute("PRAGMA journal_mode=WAL")
        self.conn.executescript(SCHEMA)
        for table, col, decl in MIGRATIONS:  # columns added after a database file was created
            try:
                self.conn.execute(f"ALTER TABLE {table} ADD COLUMN {col} {decl}")
            except sqlite3.OperationalError:
                pass
        self.lock = threading.RLock()
        self.on_change = None  # callable(table, key, cols) for streamed tables (master event stream)

    def _notify(self, table: str, key: Any, cols: Dict[str, Any]) -> None:
        cb = self.on_change
        if cb is not None and table in STREAMED:
            try:
                cb(table, key, cols)
            except Exception:  # the stream is best effort; never fail a write for it
                pass

    def _row(self, r: Optional[sqlite3.Row]) -> Optional[Dict[str, Any]]:
        if r is None:
            return None
        d = dict(r)
        for k in list(d):
            if k in JSON_COLS and isinstance(d[k], str) and d[k]:
                try:
                    d[k] = json.loads(d[k])
                except json.JSONDecodeError:
                    pass
        return d

    def execute(self, sql: str, args: Iterable[Any] = ()) -> sqlite3.Cursor:
        with self.lock:
            return self.conn.execute(sql, tuple(args))

    def one(self, sql: str, args: Iterable[Any] = ()) -> Optional[Dict[str, Any]]:
        with self.lock:
            return self._row(self.conn.execute(sql, tuple(args)).fetchone())

    def all(self, sql: str, args: Iterable[Any] = ()) -> List[Dict[str, Any]]:
        with self.lock:
            return [self._row(r) for r in self.conn.execute(sql, tuple(args)).fetchall()]  # type: ignore

    def insert(self, table: str, **cols: Any) -> int:
        keys = list(cols)
        vals = [json.dumps(v) if k in JSON_COLS and not isinstance(v, (str, bytes)) and v is not None else v
                for k, v in cols.items()]
        with self.lock:
            cur = self.conn.execute(
                f"INSERT INTO {table} ({','.join(keys)}) VALUES ({','.join('?' * len(keys))})", vals)
            rid = int(cur.lastrowid)
        self._notify(table, cols.get("id", cols.get("uuid", rid)), cols)
        return rid

    def update(self, table: str, key: str, key_val: Any, **cols: Any) -> None:
        if not cols:
            return
        sets = ",".join(f"{k}=?" for k in cols)
        vals = [json.dumps(v) if k in JSON_COLS and not isinstance(v, (str, bytes)) and v is not None else v
                for k, v in cols.items()]
        with self.lock:
            self.conn.execute(f"UPDATE {table} SET {sets} WHERE {key}=?", vals + [key_val])
        self._notify(table, key_val, cols)

    @staticmethod
    def now() -> float:
        return time.time()
