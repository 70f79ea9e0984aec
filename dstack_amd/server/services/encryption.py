"""Encryption at rest for tokens, backend credentials and secrets (reference:
``S/services/encryption/__init__.py:38-102``, ``keys/aes.py:35-68``).

AES-256-GCM through the system OpenSSL ``libcrypto`` (ctypes; the ``cryptography`` wheel is not
available), 12-byte nonce, stored as ``enc:aes:<key-name>:<base64(nonce|ciphertext|tag)>``.
Key rotation: several keys may be configured; the first encrypts, all decrypt.  ``identity`` keys
store plaintext as ``enc:identity:noname:<base64>``.
"""

from __future__ import annotations

import base64
import ctypes
import ctypes.util
import os
from dataclasses import dataclass
from typing import List, Optional


class EncryptionError(Exception):
    pass


_lib = None


def _crypto():
    global _lib
    if _lib is None:
        name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        lib = ctypes.CDLL(name)
        lib.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
        lib.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
        lib.EVP_aes_256_gcm.restype = ctypes.c_void_p
        for fn in ("EVP_EncryptInit_ex", "EVP_DecryptInit_ex"):
            getattr(lib, fn).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p,
                                         ctypes.c_char_p]
        for fn in ("EVP_EncryptUpdate", "EVP_DecryptUpdate"):
            getattr(lib, fn).argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                                         ctypes.c_char_p, ctypes.c_int]
        for fn in ("EVP_EncryptFinal_ex", "EVP_DecryptFinal_ex"):
            getattr(lib, fn).argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
        lib.EVP_CIPHER_CTX_ctrl.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        _lib = lib
    return _lib


_GCM_SET_IVLEN, _GCM_GET_TAG, _GCM_SET_TAG = 0x9, 0x10, 0x11


def aes_gcm_encrypt(key: bytes, plaintext: bytes, nonce: Optional[bytes] = None) -> bytes:
    lib = _crypto()
    nonce = nonce or os.urandom(12)
    ctx = lib.EVP_CIPHER_CTX_new()
    try:
        lib.EVP_EncryptInit_ex(ctx, lib.EVP_aes_256_gcm(), None, None, None)
        lib.EVP_CIPHER_CTX_ctrl(ctx, _GCM_SET_IVLEN, len(nonce), None)
        if lib.EVP_EncryptInit_ex(ctx, None, None, key, nonce) != 1:
            raise EncryptionError("EncryptInit failed")
        out = ctypes.create_string_buffer(len(plaintext) + 16)
        n = ctypes.c_int(0)
        lib.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), plaintext, len(plaintext))
        total = n.value
        fin = ctypes.create_string_buffer(16)
        lib.EVP_EncryptFinal_ex(ctx, fin, ctypes.byref(n))
        tag = ctypes.create_string_buffer(16)
        lib.EVP_CIPHER_CTX_ctrl(ctx, _GCM_GET_TAG, 16, tag)
        return nonce + out.raw[:total] + tag.raw
    finally:
        lib.EVP_CIPHER_CTX_free(ctx)


def aes_gcm_decrypt(key: bytes, blob: bytes) -> bytes:
    lib = _crypto()
    if len(blob) < 28:
        raise EncryptionError("ciphertext too short")
    nonce, ct, tag = blob[:12], blob[12:-16], blob[-16:]
    ctx = lib.EVP_CIPHER_CTX_new()
    try:
        lib.EVP_DecryptInit_ex(ctx, lib.EVP_aes_256_gcm(), None, None, None)
        lib.EVP_CIPHER_CTX_ctrl(ctx, _GCM_SET_IVLEN, 12, None)
        lib.EVP_DecryptInit_ex(ctx, None, None, key, nonce)
        out = ctypes.create_string_buffer(len(ct) + 16)
        n = ctypes.c_int(0)
        lib.EVP_DecryptUpdate(ctx, out, ctypes.byref(n), ct, len(ct))
        total = n.value
        tagbuf = ctypes.create_string_buffer(tag, 16)
        lib.EVP_CIPHER_CTX_ctrl(ctx, _GCM_SET_TAG, 16, tagbuf)
        fin = ctypes.create_string_buffer(16)
        if lib.EVP_DecryptFinal_ex(ctx, fin, ctypes.byref(n)) != 1:
            raise EncryptionError("authentication failed")
        return out.raw[:total]
    finally:
        lib.EVP_CIPHER_CTX_free(ctx)


@dataclass
class EncryptionKey:
    type: str  # "aes" | "identity"
    name: str
    secret: Optional[bytes] = None

    def encrypt(self, plaintext: str) -> str:
        if self.type == "identity":
            return f"enc:identity:noname:{base64.b64encode(plaintext.encode()).decode()}"
        blob = aes_gcm_encrypt(self.secret, plaintext.encode())
        return f"enc:aes:{self.name}:{base64.b64encode(blob).decode()}"

    def decrypt(self, payload: str) -> str:
        if self.type == "identity":
            return base64.b64decode(payload).decode()
        return aes_gcm_decrypt(self.secret, base64.b64decode(payload)).decode()


_IDENTITY = EncryptionKey("identity", "noname")
_keys: List[EncryptionKey] = [_IDENTITY]


def configure_keys(keys_config: Optional[list]):
    """``keys_config``: the ``encryption.keys`` list of server/config.yml."""
    global _keys
    keys = []
    for k in keys_config or []:
        if k.get("type") == "aes":
            secret = base64.b64decode(k["secret"])
            if len(secret) != 32:
                raise EncryptionError("AES key must be 32 bytes (base64)")
            keys.append(EncryptionKey("aes", k["name"], secret))
        elif k.get("type") == "identity":
            keys.append(_IDENTITY)
    keys.append(_IDENTITY)  # always able to read identity-encoded values
    _keys = keys


def encrypt(plaintext: str) -> str:
    return _keys[0].encrypt(plaintext)


def decrypt(value: str) -> str:
    if not value.startswith("enc:"):
        return value  # legacy plaintext
    _, typ, name, payload = value.split(":", 3)
    for k in _keys:
        if k.type == typ and (typ == "identity" or k.name == name):
            return k.decrypt(payload)
    raise EncryptionError(f"no encryption key {typ}:{name} configured")


def generate_aes_key() -> str:
    return base64.b64encode(os.urandom(32)).decode()
