"""Authentication primitives: HS256 JWT and bcrypt.

JWT: byte-identical to PyJWT 2.x (the reference's ``jwt.encode``,
server/raft_node.py:1713-1720): header ``{"alg":"HS256","typ":"JWT"}`` with
sorted keys and compact separators, compact payload in insertion order,
datetimes as integer epoch seconds, unpadded base64url, HMAC-SHA256.

bcrypt: the native EksBlowfish in csrc/runtime/bcrypt.cpp (GIL released),
byte-compatible with pyca/bcrypt ($2b$, cost 12 by default like
``bcrypt.gensalt()``).  Passwords are hashed to bytes; the replicated
CREATE_USER entry carries them latin-1 decoded (server/raft_node.py:1417).
"""
from __future__ import annotations

import base64
import calendar
import datetime as _dt
import hashlib
import hmac
import importlib
import json
import os
import time


class InvalidTokenError(Exception):
    pass


class ExpiredSignatureError(InvalidTokenError):
    pass


def _b64url(b: bytes) -> bytes:
    return base64.urlsafe_b64encode(b).rstrip(b"=")


def _b64url_decode(s: bytes) -> bytes:
    return base64.urlsafe_b64decode(s + b"=" * (-len(s) % 4))


class _Encoder(json.JSONEncoder):
    def default(self, o):
        if isinstance(o, _dt.datetime):
            return calendar.timegm(o.utctimetuple())
        return super().default(o)


def jwt_encode(payload: dict, secret: str, algorithm: str = "HS256") -> str:
    if algorithm != "HS256":
        raise NotImplementedError("only HS256")
    p = dict(payload)
    for k in ("exp", "iat", "nbf"):
        if isinstance(p.get(k), _dt.datetime):
            p[k] = calendar.timegm(p[k].utctimetuple())
    header = json.dumps({"alg": "HS256", "typ": "JWT"}, separators=(",", ":"), sort_keys=True)
    body = json.dumps(p, separators=(",", ":"), cls=_Encoder)
    signing = _b64url(header.encode()) + b"." + _b64url(body.encode())
    sig = hmac.new(secret.encode(), signing, hashlib.sha256).digest()
    return (signing + b"." + _b64url(sig)).decode()


def jwt_decode(token: str, secret: str, algorithms=("HS256",), leeway: float = 0.0,
               now: float | None = None) -> dict:
    try:
        tb = token.encode() if isinstance(token, str) else token
        signing, sig = tb.rsplit(b".", 1)
        h64, p64 = signing.split(b".", 1)
        header = json.loads(_b64url_decode(h64))
        payload = json.loads(_b64url_decode(p64))
        sig_b = _b64url_decode(sig)
    except Exception as e:
        raise InvalidTokenError("malformed token") from e
    if header.get("alg") not in algorithms or header.get("alg") != "HS256":
        raise InvalidTokenError("algorithm not allowed")
    want = hmac.new(secret.encode(), signing, hashlib.sha256).digest()
    if not hmac.compare_digest(want, sig_b):
        raise InvalidTokenError("signature verification failed")
    if not isinstance(payload, dict):
        raise InvalidTokenError("payload is not an object")
    if "exp" in payload:
        try:
            exp = int(payload["exp"])
        except (TypeError, ValueError) as e:
            raise InvalidTokenError("exp must be an integer") from e
        t = time.time() if now is None else now
        if exp <= t - leeway:
            raise ExpiredSignatureError("signature has expired")
    return payload


# ------------------------------------------------------------------ bcrypt
def _native():
    pkg = __name__.rsplit(".", 2)[0]
    try:
        return importlib.import_module(pkg + "._native")
    except ImportError:
        from .. import _build

        _build.build_native()
        return importlib.import_module(pkg + "._native")


def bcrypt_gensalt(rounds: int = 12, prefix: bytes = b"2b") -> bytes:
    return _native().bcrypt_gensalt(rounds, os.urandom(16), prefix.decode()[-1])


def bcrypt_hashpw(password: bytes, salt: bytes) -> bytes:
    return _native().bcrypt_hashpw(password, salt)


def bcrypt_checkpw(password: bytes, hashed: bytes) -> bool:
    if isinstance(hashed, str):
        hashed = hashed.encode("latin1")
    return _native().bcrypt_checkpw(password, hashed)
