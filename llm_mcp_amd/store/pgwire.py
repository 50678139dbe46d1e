"""Minimal PostgreSQL frontend/backend protocol v3 client (no psycopg/asyncpg
in this image).

Enough of the protocol for the control plane's store:
  * startup with TimeZone=UTC / DateStyle=ISO, auth: trust, cleartext, MD5,
    SCRAM-SHA-256;
  * extended query (Parse/Bind/Describe/Execute/Sync) with text-format
    parameters ($1..$n) and text-format results decoded by type OID;
  * simple query for multi-statement scripts (schema migrations);
  * LISTEN/NOTIFY (NotificationResponse) with a blocking ``wait_notify``;
  * a small thread-safe connection pool.

The reference reaches Postgres through pgx (core/cmd/core/main.go:53) and
LISTENs on ``job_update`` for the SSE stream (handlers.go:514-545).
"""
from __future__ import annotations

import base64
import datetime as _dt
import hashlib
import hmac
import json
import os
import queue
import re
import select
import socket
import struct
import threading
import time
from contextlib import contextmanager
from urllib.parse import parse_qs, unquote, urlparse


class PGError(Exception):
    def __init__(self, fields: dict):
        self.fields = fields
        self.code = fields.get("C", "")
        super().__init__(f"{fields.get('S', 'ERROR')} {self.code}: {fields.get('M', '')}")


def parse_dsn(dsn: str) -> dict:
    """postgres://user:pass@host:port/db?sslmode=disable  or  key=value form."""
    if "://" in dsn:
        u = urlparse(dsn)
        q = {k: v[-1] for k, v in parse_qs(u.query).items()}
        return {"host": u.hostname or "127.0.0.1", "port": u.port or 5432,
                "user": unquote(u.username or os.environ.get("PGUSER", "postgres")),
                "password": unquote(u.password or os.environ.get("PGPASSWORD", "")),
                "database": (u.path or "/").lstrip("/") or "postgres",
                "sslmode": q.get("sslmode", "prefer")}
    out = {"host": "127.0.0.1", "port": 5432, "user": "postgres", "password": "",
           "database": "postgres", "sslmode": "prefer"}
    for part in dsn.split():
        k, _, v = part.partition("=")
        out["database" if k == "dbname" else k] = v
    out["port"] = int(out["port"])
    return out


# ----------------------------------------------------------- type codecs ----
_TS_RE = re.compile(r"^(\d{4}-\d\d-\d\d[ T]\d\d:\d\d:\d\d)(?:\.(\d+))?([+-]\d\d(?::?\d\d)?)?$")


def _ts(s: str) -> float:
    # ISO DateStyle, UTC session: "2026-05-01 12:00:00.123456+00"
    if s in ("infinity", "-infinity"):
        return float("inf") if s == "infinity" else float("-inf")
    m = _TS_RE.match(s)
    if m is None:
        raise ValueError(f"unparseable timestamp {s!r}")
    frac = (m.group(2) or "").ljust(6, "0")[:6]
    tz = m.group(3) or ""
    if tz and len(tz) == 3:
        tz += ":00"
    t = _dt.datetime.fromisoformat(m.group(1) + ("." + frac if frac else "") + tz)
    if t.tzinfo is None:
        t = t.replace(tzinfo=_dt.timezone.utc)
    return t.timestamp()


_DECODE = {
    16: lambda s: s == "t",                                # bool
    20: int, 21: int, 23: int, 26: int,                    # int8/int2/int4/oid
    700: float, 701: float, 1700: float,                   # float4/float8/numeric
    114: json.loads, 3802: json.loads,                     # json/jsonb
    1184: _ts, 1114: _ts,                                  # timestamptz/timestamp
    1009: lambda s: _text_array(s), 1015: lambda s: _text_array(s),
}


def _text_array(s: str) -> list:
    body = s[1:-1]
    if not body:
        return []
    out, cur, quoted, esc, in_q = [], "", False, False, False
    for ch in body:
        if esc:
            cur += ch
            esc = False
        elif ch == "\\":
            esc = True
        elif ch == '"':
            in_q = not in_q
            quoted = True
        elif ch == "," and not in_q:
            out.append(cur if quoted or cur != "NULL" else None)
            cur, quoted = "", False
        else:
            cur += ch
    out.append(cur if quoted or cur != "NULL" else None)
    return out


def encode_param(v) -> bytes | None:
    if v is None:
        return None
    if isinstance(v, bool):
        return b"t" if v else b"f"
    if isinstance(v, (int, float)):
        return repr(v).encode() if isinstance(v, float) else str(v).encode()
    if isinstance(v, (dict,)):
        return json.dumps(v).encode()
    if isinstance(v, (list, tuple)):
        # text[] literal
        items = []
        for x in v:
            if x is None:
                items.append("NULL")
            else:
                items.append('"' + str(x).replace("\\", "\\\\").replace('"', '\\"') + '"')
        return ("{" + ",".join(items) + "}").encode()
    if isinstance(v, bytes):
        return v
    return str(v).encode()


# ------------------------------------------------------------ connection ----
class Connection:
    def __init__(self, dsn: str | dict, timeout: float = 10.0, application_name: str = "lmx"):
        self.params = parse_dsn(dsn) if isinstance(dsn, str) else dict(dsn)
        if self.params.get("sslmode") in ("require", "verify-ca", "verify-full"):
            raise PGError({"M": "TLS to Postgres is not supported by the in-tree client; "
                                "use sslmode=disable on a private network"})
        self.sock = socket.create_connection((self.params["host"], int(self.params["port"])),
                                             timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.buf = b""
        self.notifications: list[tuple[str, str]] = []
        self.server_params: dict[str, str] = {}
        self.tx_status = "I"
        self._startup(application_name)
        self.sock.settimeout(None)

    # ---- framing
    def _send(self, typ: bytes, body: bytes = b""):
        self.sock.sendall(typ + struct.pack("!I", len(body) + 4) + body)

    def _recv_exact(self, n: int) -> bytes:
        while len(self.buf) < n:
            chunk = self.sock.recv(max(65536, n - len(self.buf)))
            if not chunk:
                raise ConnectionError("postgres closed the connection")
            self.buf += chunk
        out, self.buf = self.buf[:n], self.buf[n:]
        return out

    def _read(self) -> tuple[bytes, bytes]:
        hdr = self._recv_exact(5)
        n = struct.unpack("!I", hdr[1:])[0]
        return hdr[:1], self._recv_exact(n - 4)

    @staticmethod
    def _fields(body: bytes) -> dict:
        out = {}
        for part in body.split(b"\x00"):
            if part:
                out[chr(part[0])] = part[1:].decode("utf-8", "replace")
        return out

    def _common(self, typ: bytes, body: bytes) -> bool:
        """Handle asynchronous messages; True if consumed."""
        if typ == b"A":
            pid = struct.unpack("!I", body[:4])[0]
            ch, _, rest = body[4:].partition(b"\x00")
            payload = rest.split(b"\x00")[0]
            self.notifications.append((ch.decode(), payload.decode()))
            return True
        if typ == b"N":
            return True
        if typ == b"S":
            k, v = body.rstrip(b"\x00").split(b"\x00", 1)
            self.server_params[k.decode()] = v.decode()
            return True
        return False

    # ---- startup / auth
    def _startup(self, app: str):
        p = self.params
        kv = [("user", p["user"]), ("database", p["database"]), ("application_name", app),
              ("TimeZone", "UTC"), ("DateStyle", "ISO")]
        body = struct.pack("!I", 196608) + b"".join(
            k.encode() + b"\x00" + v.encode() + b"\x00" for k, v in kv) + b"\x00"
        self.sock.sendall(struct.pack("!I", len(body) + 4) + body)
        scram = None
        while True:
            typ, body = self._read()
            if typ == b"R":
                code = struct.unpack("!I", body[:4])[0]
                if code == 0:
                    continue
                if code == 3:
                    self._send(b"p", p["password"].encode() + b"\x00")
                elif code == 5:
                    salt = body[4:8]
                    inner = hashlib.md5(p["password"].encode() + p["user"].encode()).hexdigest()
                    outer = hashlib.md5(inner.encode() + salt).hexdigest()
                    self._send(b"p", b"md5" + outer.encode() + b"\x00")
                elif code == 10:
                    mechs = [m for m in body[4:].split(b"\x00") if m]
                    if b"SCRAM-SHA-256" not in mechs:
                        raise PGError({"M": f"unsupported SASL mechanisms {mechs}"})
                    scram = _Scram(p["password"])
                    first = scram.client_first().encode()
                    self._send(b"p", b"SCRAM-SHA-256\x00" + struct.pack("!I", len(first)) + first)
                elif code == 11:
                    self._send(b"p", scram.client_final(body[4:].decode()).encode())
                elif code == 12:
                    scram.verify(body[4:].decode())
                else:
                    raise PGError({"M": f"unsupported auth method {code}"})
            elif typ == b"E":
                raise PGError(self._fields(body))
            elif typ == b"K":
                self.backend_pid = struct.unpack("!I", body[:4])[0]
            elif typ == b"Z":
                self.tx_status = body.decode()
                return
            else:
                self._common(typ, body)

    # ---- queries
    def execute(self, sql: str, params: tuple | list = ()) -> tuple[list[dict], str]:
        """Extended-protocol query; returns (rows as dicts, command tag)."""
        vals = [encode_param(v) for v in params]
        parse = b"\x00" + sql.encode() + b"\x00" + struct.pack("!H", 0)
        bind = [b"\x00\x00", struct.pack("!HH", 0, len(vals))]
        for v in vals:
            bind.append(struct.pack("!i", -1) if v is None else struct.pack("!I", len(v)) + v)
        bind.append(struct.pack("!H", 0))
        msg = (b"P" + struct.pack("!I", len(parse) + 4) + parse
               + b"B" + struct.pack("!I", len(b"".join(bind)) + 4) + b"".join(bind)
               + b"D" + struct.pack("!I", 6) + b"P\x00"
               + b"E" + struct.pack("!I", 9) + b"\x00" + struct.pack("!I", 0)
               + b"S" + struct.pack("!I", 4))
        self.sock.sendall(msg)
        return self._collect()

    def simple(self, sql: str) -> tuple[list[dict], str]:
        self._send(b"Q", sql.encode() + b"\x00")
        return self._collect()

    def _collect(self):
        cols: list[tuple[str, int]] = []
        rows: list[dict] = []
        tag, err = "", None
        while True:
            typ, body = self._read()
            if typ == b"T":
                n = struct.unpack("!H", body[:2])[0]
                off, cols = 2, []
                for _ in range(n):
                    end = body.index(b"\x00", off)
                    name = body[off:end].decode()
                    oid = struct.unpack("!I", body[end + 7:end + 11])[0]
                    cols.append((name, oid))
                    off = end + 19
            elif typ == b"D":
                n = struct.unpack("!H", body[:2])[0]
                off, row = 2, {}
                for i in range(n):
                    ln = struct.unpack("!i", body[off:off + 4])[0]
                    off += 4
                    name, oid = cols[i]
                    if ln < 0:
                        row[name] = None
                        continue
                    s = body[off:off + ln].decode("utf-8")
                    off += ln
                    dec = _DECODE.get(oid)
                    row[name] = dec(s) if dec else s
                rows.append(row)
            elif typ == b"C":
                tag = body.rstrip(b"\x00").decode()
            elif typ == b"E":
                err = PGError(self._fields(body))
            elif typ == b"Z":
                self.tx_status = body.decode()
                if err is not None:
                    raise err
                return rows, tag
            elif typ in (b"1", b"2", b"n", b"I", b"s"):
                continue
            else:
                self._common(typ, body)

    def query(self, sql: str, *params) -> list[dict]:
        return self.execute(sql, params)[0]

    def one(self, sql: str, *params) -> dict | None:
        r = self.execute(sql, params)[0]
        return r[0] if r else None

    def scalar(self, sql: str, *params):
        r = self.one(sql, *params)
        return None if r is None else next(iter(r.values()))

    def rowcount(self, sql: str, *params) -> int:
        tag = self.execute(sql, params)[1]
        try:
            return int(tag.rsplit(" ", 1)[-1])
        except ValueError:
            return 0

    @contextmanager
    def transaction(self):
        self.simple("BEGIN")
        try:
            yield self
        except BaseException:
            self.simple("ROLLBACK")
            raise
        else:
            self.simple("COMMIT")

    # ---- LISTEN/NOTIFY
    def listen(self, channel: str):
        self.simple(f'LISTEN "{channel}"')

    def wait_notify(self, timeout: float) -> list[tuple[str, str]]:
        deadline = time.monotonic() + timeout
        while not self.notifications:
            left = deadline - time.monotonic()
            if left <= 0:
                break
            if not self.buf:
                r, _, _ = select.select([self.sock], [], [], left)
                if not r:
                    break
                chunk = self.sock.recv(65536)
                if not chunk:
                    raise ConnectionError("postgres closed the connection")
                self.buf += chunk
            while len(self.buf) >= 5:
                n = struct.unpack("!I", self.buf[1:5])[0]
                if len(self.buf) < n + 1:
                    break
                typ, body = self._read()
                self._common(typ, body)
        out, self.notifications = self.notifications, []
        return out

    def close(self):
        try:
            self._send(b"X")
        except OSError:
            pass
        self.sock.close()


class _Scram:
    def __init__(self, password: str):
        self.pw = password.encode()
        self.nonce = base64.b64encode(os.urandom(18)).decode()

    def client_first(self) -> str:
        self.first_bare = f"n=,r={self.nonce}"
        return "n,," + self.first_bare

    def client_final(self, server_first: str) -> str:
        a = dict(x.split("=", 1) for x in server_first.split(","))
        if not a["r"].startswith(self.nonce):
            raise PGError({"M": "SCRAM nonce mismatch"})
        salted = hashlib.pbkdf2_hmac("sha256", self.pw, base64.b64decode(a["s"]), int(a["i"]))
        ckey = hmac.new(salted, b"Client Key", hashlib.sha256).digest()
        stored = hashlib.sha256(ckey).digest()
        without_proof = f"c=biws,r={a['r']}"
        self.auth_msg = f"{self.first_bare},{server_first},{without_proof}".encode()
        sig = hmac.new(stored, self.auth_msg, hashlib.sha256).digest()
        proof = bytes(x ^ y for x, y in zip(ckey, sig))
        self.server_key = hmac.new(salted, b"Server Key", hashlib.sha256).digest()
        return f"{without_proof},p={base64.b64encode(proof).decode()}"

    def verify(self, server_final: str):
        a = dict(x.split("=", 1) for x in server_final.split(","))
        want = hmac.new(self.server_key, self.auth_msg, hashlib.sha256).digest()
        if base64.b64decode(a.get("v", "")) != want:
            raise PGError({"M": "SCRAM server signature mismatch"})


class Pool:
    """Thread-safe pool; ``with pool.conn() as c: c.query(...)``."""

    def __init__(self, dsn: str, size: int = 8):
        self.dsn, self.size = dsn, size
        self._free: queue.LifoQueue = queue.LifoQueue()
        self._n = 0
        self._lock = threading.Lock()

    @contextmanager
    def conn(self):
        c = None
        try:
            c = self._free.get_nowait()
        except queue.Empty:
            with self._lock:
                make = self._n < self.size
                if make:
                    self._n += 1
            if make:
                try:
                    c = Connection(self.dsn)
                except BaseException:
                    with self._lock:
                        self._n -= 1
                    raise
            else:
                c = self._free.get(timeout=30)
        broken = False
        try:
            yield c
        except (ConnectionError, OSError):
            broken = True
            raise
        finally:
            if broken or c.tx_status == "E":
                try:
                    c.close()
                except Exception:
                    pass
                with self._lock:
                    self._n -= 1
            else:
                self._free.put(c)

    def close(self):
        while True:
            try:
                self._free.get_nowait().close()
            except queue.Empty:
                return
