"""Authentication for the REST server: HTTP Basic against a Jetty
HashLoginService realm file (the reference's `-hash_login -login_conf
realm.properties`, water/webserver + h2o-jetty-9 Jetty9Helper), optional TLS
via PEM certificate / key (the reference uses a JKS keystore, `-jks`).

Realm file lines: ``username: password[,role ...]`` where password is plain
text, ``MD5:<hex digest>`` or Jetty-obfuscated ``OBF:...``; ``#`` comments.
"""
from __future__ import annotations

import base64
import hashlib
import hmac


def deobfuscate(s: str) -> str:
    """Jetty's Password.deobfuscate for OBF: strings (groups of 4 base-36
    digits, or 'U' + 5 digits for code points above 255)."""
    if s.startswith("OBF:"):
        s = s[4:]
    out = []
    i = 0
    while i < len(s):
        if s[i] == "U":
            i += 1
            l = int(s[i:i + 5], 36)
            i += 5
            out.append(chr(l >> 8))
        else:
            x = s[i:i + 4]
            i += 4
            ii = int(x, 36)
            i1, i2 = ii // 256, ii % 256
            out.append(chr((i1 + i2 - 254) // 2))
    return "".join(out)


def load_realm(path: str) -> dict[str, str]:
    """user -> stored credential from a HashLoginService properties file."""
    users = {}
    with open(path, encoding="utf-8") as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#") or ":" not in line:
                continue
            user, rest = line.split(":", 1)
            cred = rest.strip().split(",")[0].strip()
            users[user.strip()] = cred
    return users


def check_password(stored: str, given: str) -> bool:
    if stored.startswith("MD5:"):
        return hmac.compare_digest(stored[4:].lower(), hashlib.md5(given.encode()).hexdigest())
    if stored.startswith("OBF:"):
        stored = deobfuscate(stored)
    return hmac.compare_digest(stored.encode(), given.encode())


def basic_auth_middleware(app, users: dict[str, str], realm: str = "h2o"):
    """ASGI middleware: every HTTP request needs valid Basic credentials."""

    async def mw(scope, receive, send):
        if scope["type"] != "http":
            return await app(scope, receive, send)
        hdr = dict(scope.get("headers") or []).get(b"authorization", b"").decode("latin-1")
        ok = False
        if hdr.lower().startswith("basic "):
            try:
                user, _, pw = base64.b64decode(hdr[6:].strip()).decode("utf-8").partition(":")
                ok = user in users and check_password(users[user], pw)
            except (ValueError, UnicodeDecodeError):
                ok = False
        if ok:
            return await app(scope, receive, send)
        body = b'{"http_status": 401, "msg": "Unauthorized"}'
        await send({"type": "http.response.start", "status": 401,
                    "headers": [(b"content-type", b"application/json"),
                                (b"www-authenticate", f'Basic realm="{realm}"'.encode()),
                                (b"content-length", str(len(body)).encode())]})
        await send({"type": "http.response.body", "body": body})
    return mw
