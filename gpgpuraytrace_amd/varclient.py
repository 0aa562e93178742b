"""Live-tweak client (variableclient/VariableManager.cs) for the VariableManager protocol that
rt_varmgr_start serves (Common/VariableManager.cpp:76-83):

    server -> client   [1][name len:1][name][type len:1][type][size:2 LE][data]   add
                       [0][name len:1][name]                                     remove
                       [2]                                                       remove all
    client -> server   [name len:1][name][data]                                  write

Variables decode by their HLSL type name (float, float2, float3, float4 -> float32 arrays),
as the C# client's Native._<type> structs do.
"""
import socket
import struct

import numpy as np

PORT = 10666  # VariableManager.cs / VariableManager.cpp:131


class VariableClient:
    def __init__(self, address="127.0.0.1", port=PORT, timeout=5.0):
        self.sock = socket.create_connection((address, port), timeout=timeout)
        self.variables = {}  # name -> (type, raw bytes)
        self._buf = b""

    def close(self):
        self.sock.close()

    def _read(self, n):
        while len(self._buf) < n:
            chunk = self.sock.recv(65536)
            if not chunk:
                raise ConnectionError("server closed the connection")
            self._buf += chunk
        out, self._buf = self._buf[:n], self._buf[n:]
        return out

    def poll(self):
        """Read one server packet and apply it; returns its kind ('add', 'remove', 'clear')."""
        kind = self._read(1)[0]
        if kind == 1:
            name = self._read(self._read(1)[0]).decode("ascii")
            typ = self._read(self._read(1)[0]).decode("ascii")
            size = struct.unpack("<H", self._read(2))[0]
            self.variables[name] = (typ, self._read(size))
            return "add"
        if kind == 0:
            self.variables.pop(self._read(self._read(1)[0]).decode("ascii"), None)
            return "remove"
        if kind == 2:
            self.variables.clear()
            return "clear"
        return "unknown"

    def value(self, name):
        typ, raw = self.variables[name]
        return np.frombuffer(raw, np.float32).copy() if typ.startswith("float") else raw

    def send(self, name, value):
        """Write a variable: [name len][name][data], data = the value as float32 bytes."""
        data = np.asarray(value, np.float32).tobytes() if not isinstance(value, (bytes, bytearray)) else bytes(value)
        nm = name.encode("ascii")
        self.sock.sendall(bytes([len(nm)]) + nm + data)
