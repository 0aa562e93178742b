"""VariableManager live-tweak protocol on the CPU: the native server
(rt_varmgr_*, no GPU needed while no compute is registered) against the Python client, and the
client's packet decoding against a scripted server."""
import socket
import struct
import threading

import numpy as np
import pytest

from gpgpuraytrace_amd import varclient as VC


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_client_decodes_add_remove_clear():
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]
    got = {}

    def serve():
        c, _ = srv.accept()
        add = bytes([1, 12]) + b"SunDirection" + bytes([6]) + b"float3" + struct.pack("<H", 12) + \
            np.array([0.1, -0.9, 0.1], np.float32).tobytes()
        c.sendall(add + bytes([1, 1]) + b"k" + bytes([5]) + b"float" + struct.pack("<H", 4) +
                  np.float32(2.5).tobytes() + bytes([0, 1]) + b"k" + bytes([2]))
        got["write"] = c.recv(64)
        c.close()

    t = threading.Thread(target=serve)
    t.start()
    cl = VC.VariableClient("127.0.0.1", port)
    assert cl.poll() == "add" and cl.poll() == "add"
    assert cl.value("SunDirection").tolist() == pytest.approx([0.1, -0.9, 0.1]) and cl.value("k")[0] == 2.5
    assert cl.poll() == "remove" and set(cl.variables) == {"SunDirection"}
    assert cl.poll() == "clear" and not cl.variables
    cl.send("SunDirection", [0.0, -1.0, 0.0])
    t.join()
    cl.close()
    srv.close()
    assert got["write"] == bytes([12]) + b"SunDirection" + np.array([0, -1, 0], np.float32).tobytes()


def test_native_server_empty_registry_and_unknown_variable():
    import gpgpuraytrace_amd as G
    port = _free_port()
    G.VariableManager.start(port)
    try:
        assert G.VariableManager.count() == 0
        with pytest.raises(Exception):
            G.VariableManager.start(port)  # already running
        cl = VC.VariableClient("127.0.0.1", port)
        cl.send("Nope", b"\x00" * 4)  # VariableManager.cpp:172-177: unknown variable closes the client
        cl.sock.settimeout(5.0)
        try:
            assert cl.sock.recv(16) == b""
        except ConnectionResetError:  # closed with the unread payload still queued
            pass
        cl.close()
    finally:
        G.VariableManager.stop()
    G.VariableManager.stop()  # idempotent


def test_native_server_survives_malformed_clients():
    """Untrusted bytes on the live-tweak port (VariableManager.cpp:144-185 reads a name length byte,
    the name and the variable's bytes): random and truncated packets, zero-length and maximal names,
    clients that vanish mid-packet.  The server must close such clients and keep serving; run under
    ASan + UBSan by scripts/sanitize_cpu.sh."""
    import gpgpuraytrace_amd as G
    rng = np.random.default_rng(7)
    port = _free_port()
    G.VariableManager.start(port)
    try:
        payloads = [b"", bytes([0]), bytes([255]), bytes([255]) + b"A" * 255, bytes([200]) + b"x" * 10,
                    bytes([4]) + b"Nope", bytes([12]) + b"SunDirection"]
        payloads += [rng.integers(0, 256, size=int(n), dtype=np.uint8).tobytes() for n in rng.integers(1, 600, 24)]
        for p in payloads:
            s = socket.create_connection(("127.0.0.1", port), timeout=5.0)
            s.sendall(p)
            s.close()
        # still serving: a well-formed client is accepted and gets its (empty) registry
        cl = VC.VariableClient("127.0.0.1", port)
        cl.sock.settimeout(2.0)
        cl.close()
        assert G.VariableManager.count() == 0
    finally:
        G.VariableManager.stop()
