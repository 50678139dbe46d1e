"""A scripted PostgreSQL v3 protocol server for testing the in-tree client
(no Postgres server exists in this image).  It speaks the real framing:
startup, MD5 / SCRAM-SHA-256 / trust auth, simple and extended query,
RowDescription/DataRow/CommandComplete/ErrorResponse/ReadyForQuery and
NotificationResponse.  Query results come from a ``handler(sql, params)``
callback returning ``(columns, rows, tag)`` with columns = [(name, oid)]."""
from __future__ import annotations

import base64
import hashlib
import hmac
import os
import socket
import struct
import threading


class FakePG:
    def __init__(self, handler, auth: str = "md5", user: str = "lmx", password: str = "pw"):
        self.handler, self.auth, self.user, self.password = handler, auth, user, password
        self.sock = socket.socket()
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(16)
        self.port = self.sock.getsockname()[1]
        self.log: list[tuple[str, list]] = []
        self.listeners: list = []
        self._stop = False
        threading.Thread(target=self._accept, daemon=True).start()

    @property
    def dsn(self):
        return f"postgres://{self.user}:{self.password}@127.0.0.1:{self.port}/lmx?sslmode=disable"

    def close(self):
        self._stop = True
        self.sock.close()

    def notify(self, channel: str, payload: str):
        for c in list(self.listeners):
            try:
                body = struct.pack("!I", 1) + channel.encode() + b"\0" + payload.encode() + b"\0"
                c.sendall(b"A" + struct.pack("!I", len(body) + 4) + body)
            except OSError:
                pass

    # ------------------------------------------------------------------ io --
    def _accept(self):
        while not self._stop:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    @staticmethod
    def _recv(c, n):
        b = b""
        while len(b) < n:
            x = c.recv(n - len(b))
            if not x:
                raise ConnectionError
            b += x
        return b

    def _msg(self, c):
        h = self._recv(c, 5)
        return h[:1], self._recv(c, struct.unpack("!I", h[1:])[0] - 4)

    @staticmethod
    def _send(c, typ, body=b""):
        c.sendall(typ + struct.pack("!I", len(body) + 4) + body)

    def _serve(self, c):
        try:
            n = struct.unpack("!I", self._recv(c, 4))[0]
            body = self._recv(c, n - 4)
            kv = body[4:].split(b"\0")
            params = dict(zip(kv[0::2], kv[1::2]))
            assert params[b"user"].decode() == self.user
            if not self._authenticate(c):
                return
            self._send(c, b"S", b"TimeZone\0UTC\0")
            self._send(c, b"K", struct.pack("!II", 42, 7))
            self._send(c, b"Z", b"I")
            pending = None
            while True:
                typ, body = self._msg(c)
                if typ == b"X":
                    return
                if typ == b"Q":
                    self._run(c, body.rstrip(b"\0").decode(), [], describe=True)
                    self._send(c, b"Z", b"I")
                elif typ == b"P":
                    parts = body.split(b"\0")
                    pending = {"sql": parts[1].decode(), "params": [], "error": None}
                    self._send(c, b"1")
                elif typ == b"B":
                    off = body.index(b"\0") + 1
                    off = body.index(b"\0", off) + 1
                    nfmt = struct.unpack("!H", body[off:off + 2])[0]
                    off += 2 + 2 * nfmt
                    np_ = struct.unpack("!H", body[off:off + 2])[0]
                    off += 2
                    vals = []
                    for _ in range(np_):
                        ln = struct.unpack("!i", body[off:off + 4])[0]
                        off += 4
                        if ln < 0:
                            vals.append(None)
                        else:
                            vals.append(body[off:off + ln].decode())
                            off += ln
                    pending["params"] = vals
                    self._send(c, b"2")
                elif typ == b"D":
                    pass
                elif typ == b"E":
                    self._run(c, pending["sql"], pending["params"], describe=True)
                elif typ == b"S":
                    self._send(c, b"Z", b"I")
        except (ConnectionError, OSError):
            pass
        finally:
            if c in self.listeners:
                self.listeners.remove(c)
            c.close()

    def _run(self, c, sql, params, describe):
        self.log.append((sql, params))
        if sql.strip().upper().startswith("LISTEN"):
            self.listeners.append(c)
            self._send(c, b"C", b"LISTEN\0")
            return
        try:
            cols, rows, tag = self.handler(sql, params)
        except Exception as e:  # noqa: BLE001 -- becomes an ErrorResponse
            body = b"SERROR\0C42000\0M" + str(e).encode() + b"\0\0"
            self._send(c, b"E", body)
            return
        if cols:
            desc = struct.pack("!H", len(cols))
            for name, oid in cols:
                desc += name.encode() + b"\0" + struct.pack("!IhIhih", 0, 0, oid, -1, -1, 0)
            self._send(c, b"T", desc)
            for r in rows:
                d = struct.pack("!H", len(r))
                for v in r:
                    if v is None:
                        d += struct.pack("!i", -1)
                    else:
                        b = str(v).encode()
                        d += struct.pack("!I", len(b)) + b
                self._send(c, b"D", d)
        elif describe:
            self._send(c, b"n")
        self._send(c, b"C", tag.encode() + b"\0")

    # ---------------------------------------------------------------- auth --
    def _authenticate(self, c) -> bool:
        if self.auth == "trust":
            self._send(c, b"R", struct.pack("!I", 0))
            return True
        if self.auth == "md5":
            salt = os.urandom(4)
            self._send(c, b"R", struct.pack("!I", 5) + salt)
            _, body = self._msg(c)
            inner = hashlib.md5((self.password + self.user).encode()).hexdigest()
            want = "md5" + hashlib.md5(inner.encode() + salt).hexdigest()
            if body.rstrip(b"\0").decode() != want:
                self._send(c, b"E", b"SFATAL\0C28P01\0Mpassword authentication failed\0\0")
                return False
            self._send(c, b"R", struct.pack("!I", 0))
            return True
        # SCRAM-SHA-256 (RFC 5802 / 7677), server side
        self._send(c, b"R", struct.pack("!I", 10) + b"SCRAM-SHA-256\0\0")
        _, body = self._msg(c)
        mech_end = body.index(b"\0")
        ln = struct.unpack("!I", body[mech_end + 1:mech_end + 5])[0]
        first = body[mech_end + 5:mech_end + 5 + ln].decode()
        first_bare = first.split(",", 2)[2]
        cnonce = dict(x.split("=", 1) for x in first_bare.split(","))["r"]
        salt, iters = os.urandom(16), 4096
        snonce = cnonce + base64.b64encode(os.urandom(18)).decode()
        server_first = f"r={snonce},s={base64.b64encode(salt).decode()},i={iters}"
        self._send(c, b"R", struct.pack("!I", 11) + server_first.encode())
        _, body = self._msg(c)
        final = body.decode()
        attrs = dict(x.split("=", 1) for x in final.split(","))
        without_proof = final[:final.rindex(",p=")]
        salted = hashlib.pbkdf2_hmac("sha256", self.password.encode(), salt, iters)
        ckey = hmac.new(salted, b"Client Key", hashlib.sha256).digest()
        stored = hashlib.sha256(ckey).digest()
        auth_msg = f"{first_bare},{server_first},{without_proof}".encode()
        sig = hmac.new(stored, auth_msg, hashlib.sha256).digest()
        proof = base64.b64decode(attrs["p"])
        if hashlib.sha256(bytes(a ^ b for a, b in zip(proof, sig))).digest() != stored:
            self._send(c, b"E", b"SFATAL\0C28P01\0MSCRAM authentication failed\0\0")
            return False
        skey = hmac.new(salted, b"Server Key", hashlib.sha256).digest()
        v = base64.b64encode(hmac.new(skey, auth_msg, hashlib.sha256).digest()).decode()
        self._send(c, b"R", struct.pack("!I", 12) + f"v={v}".encode())
        self._send(c, b"R", struct.pack("!I", 0))
        return True
