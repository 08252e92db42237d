"""Launcher and line-protocol client of ``lsmck_server`` (csrc/lsmck_server.cpp),
the loopback server of the reference (src/server.rs; protocol src/command.rs).

``Server(base, ...)`` starts the binary, waits for its start-up (Db::load: the
GPU tree verify and WAL replay) and exposes the JSON it reports (later events,
such as each compaction tick's re-verify, through ``wait_event``); ``Client``
speaks the newline-terminated protocol: ``insert k v`` / ``update k v`` ->
"ok", ``delete k`` -> "ok", ``get k`` -> the value or "<k> not found".
"""
import collections
import json
import os
import queue
import signal
import socket
import subprocess
import threading
import time

BIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lsmck_server")


class ServerExited(RuntimeError):
    def __init__(self, rc, stderr):
        super().__init__(f"lsmck_server exited with {rc}: {stderr.strip()[-500:]}")
        self.rc = rc
        self.stderr = stderr


class Server:
    def __init__(self, base, port=0, memtable_limit=4096, device=0, timeout=600, exit_after_load=False,
                 compact_interval_ms=None, index_threads=None):
        if not os.path.exists(BIN):
            raise FileNotFoundError(f"{BIN} is not built (make -C lsm_storage_engine_amd/csrc)")
        cmd = [BIN, "--base", str(base), "--port", str(port), "--memtable-limit", str(memtable_limit),
               "--device", str(device)]
        if exit_after_load:
            cmd.append("--exit-after-load")
        if compact_interval_ms is not None:  # the server's default is the reference's 10 s tick
            cmd += ["--compact-interval", str(int(compact_interval_ms))]
        if index_threads is not None:  # Db::load's index-loading threads (A/B)
            cmd += ["--index-threads", str(int(index_threads))]
        self.proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        # stderr is drained on its own thread into a bounded tail: an undrained
        # pipe fills at 64 KiB (LSMCK_TREE_TRACE prints a line per round) and
        # the server would block in write(2) in the middle of a load
        self._err = collections.deque(maxlen=256)
        self._err_thread = threading.Thread(target=lambda: [self._err.append(x) for x in iter(self.proc.stderr.readline, "")],
                                            daemon=True)
        self._err_thread.start()
        self.loaded = None
        self.port = None
        # the event lines come through a reader thread (select() on a buffered
        # pipe misses lines already read into the buffer)
        self._lines = lines = queue.Queue()
        threading.Thread(target=lambda: [lines.put(x) for x in iter(self.proc.stdout.readline, "")] + [lines.put("")],
                         daemon=True).start()
        deadline = time.time() + timeout
        while self.port is None and not (exit_after_load and self.loaded):
            try:
                line = lines.get(timeout=max(0.01, deadline - time.time()))
            except queue.Empty:
                self.kill()
                raise TimeoutError("lsmck_server did not start")
            if not line:
                rc = self.proc.wait()
                raise ServerExited(rc, self.stderr_tail())
            ev = json.loads(line)
            if ev["event"] == "loaded":
                self.loaded = ev
            elif ev["event"] == "listening":
                self.port = ev["port"]
        if exit_after_load:
            self.proc.wait(timeout=60)

    def wait_event(self, kind, timeout=120):
        """The next JSON event line of this kind the server prints after start-up
        (e.g. "compact" / "compact_failed": a compaction tick's re-verify)."""
        deadline = time.time() + timeout
        while True:
            try:
                line = self._lines.get(timeout=max(0.01, deadline - time.time()))
            except queue.Empty:
                raise TimeoutError(f"no {kind!r} event from lsmck_server")
            if not line:
                raise ServerExited(self.proc.wait(), self.stderr_tail())
            ev = json.loads(line)
            if ev["event"] == kind:
                return ev

    def drain_events(self, kind):
        """Every event line of this kind printed so far (no waiting)."""
        out = []
        while True:
            try:
                line = self._lines.get_nowait()
            except queue.Empty:
                return out
            if line and json.loads(line)["event"] == kind:
                out.append(json.loads(line))

    def wait_stderr(self, text, timeout=10.0):
        """The stderr lines once one contains `text` (read by a drain thread,
        so a line written before an event on stdout can arrive after it)."""
        t_end = time.monotonic() + timeout
        while text not in self.stderr_tail() and time.monotonic() < t_end and self.proc.poll() is None:
            time.sleep(0.02)
        return self.stderr_tail()

    def stderr_tail(self):
        """The last lines the server wrote to stderr (all of them once it has exited)."""
        if self.proc.poll() is not None:
            self._err_thread.join(timeout=5)
        return "".join(self._err)

    def kill(self):
        """SIGKILL: no flush, no clean shutdown (a crash)."""
        if self.proc.poll() is None:
            self.proc.send_signal(signal.SIGKILL)
            self.proc.wait()

    def client(self):
        return Client(self.port)


class Client:
    def __init__(self, port, host="127.0.0.1"):
        self.sock = socket.create_connection((host, port))
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.buf = b""

    def _line(self):
        while b"\n" not in self.buf:
            chunk = self.sock.recv(1 << 16)
            if not chunk:
                raise ConnectionError("server closed the connection")
            self.buf += chunk
        line, self.buf = self.buf.split(b"\n", 1)
        return line

    def call(self, *args):
        self.sock.sendall(b" ".join(a if isinstance(a, bytes) else str(a).encode() for a in args) + b"\n")
        return self._line()

    def pipeline(self, commands):
        """Send many command lines at once, then read one response per line."""
        self.sock.sendall(b"".join(c + b"\n" for c in commands))
        return [self._line() for _ in commands]

    def close(self):
        self.sock.close()
