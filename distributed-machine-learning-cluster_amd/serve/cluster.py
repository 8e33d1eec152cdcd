"""Local multi-node cluster launcher and REPL driver for ``dmlc-node``.

The reference could only run one node per host (ports and hostnames are
constants: src/membership.rs:64, src/services.rs:26-32) and was tested by
hand on 10 VMs (CS425MP4Report.pdf). Every port/period here is a flag, so N
nodes run as N processes on one machine; this module starts them, feeds
their stdin REPL (same verbs as src/main.rs:85-338) and matches their stdout.
"""
from __future__ import annotations

import os
import queue
import re
import signal
import subprocess
import threading
import time

from .. import REPO_ROOT

NODE_BIN = os.path.join(REPO_ROOT, "build", "bin", "dmlc-node")


class NodeProcess:
    def __init__(self, port: int, leaders: list[str], workdir: str, labels: str, dataset: str = "",
                 models: str = "", executor: str = "cpu", host: str = "127.0.0.1", fast: bool = True,
                 extra: list[str] | None = None, env: dict | None = None, binary: str | None = None):
        self.port = port
        self.address = f"{host}:{port}"
        os.makedirs(workdir, exist_ok=True)
        args = [binary or os.environ.get("DMLC_NODE_BIN", NODE_BIN), "--host", host, "--port", str(port), "--leaders", ",".join(leaders),
                "--workdir", workdir, "--labels", labels, "--executor", executor, "--ack"]
        if dataset:
            args += ["--dataset", dataset]
        if models:
            args += ["--models", models]
        if fast:
            args += ["--ping-ms", "200", "--detect-ms", "200", "--fail-ms", "1200", "--bg-ms", "500"]
        args += extra or []
        e = dict(os.environ)
        e.setdefault("OMP_NUM_THREADS", "2")
        e.update(env or {})
        self.proc = subprocess.Popen(args, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                     text=True, bufsize=1, env=e, start_new_session=True)
        self.lines: list[str] = []
        self._q: queue.Queue[str] = queue.Queue()
        self._cursor = 0
        self._lock = threading.Lock()
        self._t = threading.Thread(target=self._reader, daemon=True)
        self._t.start()

    def _reader(self):
        for line in self.proc.stdout:
            with self._lock:
                self.lines.append(line.rstrip("\n"))

    def send(self, line: str) -> None:
        try:
            self.proc.stdin.write(line + "\n")
            self.proc.stdin.flush()
        except BrokenPipeError as e:  # the node exited: say how, with its last output
            rc = self.proc.wait(timeout=5)
            raise RuntimeError(f"node {self.address} exited (rc {rc}) before {line!r}; output:\n"
                               f"{self.output()[-4000:]}") from e

    def mark(self) -> int:
        with self._lock:
            return len(self.lines)

    def output(self, since: int = 0) -> str:
        with self._lock:
            return "\n".join(self.lines[since:])

    def expect(self, pattern: str, timeout: float = 10.0, since: int | None = None) -> re.Match:
        start = self._cursor if since is None else since
        rx = re.compile(pattern, re.M)
        deadline = time.time() + timeout
        while time.time() < deadline:
            text = self.output(start)
            m = rx.search(text)
            if m:
                return m
            if self.proc.poll() is not None:
                break
            time.sleep(0.05)
        raise TimeoutError(f"node {self.address}: /{pattern}/ not seen; output since {start}:\n{self.output(start)}")

    def run(self, line: str, pattern: str, timeout: float = 20.0) -> re.Match:
        since = self.mark()
        self.send(line)
        return self.expect(pattern, timeout, since)

    def cmd(self, line: str, timeout: float = 30.0) -> str:
        """Run one REPL command and return its complete output (the node
        runs with --ack and prints <<done>> after every command)."""
        since = self.mark()
        self.send(line)
        deadline = time.time() + timeout
        while time.time() < deadline:
            with self._lock:
                chunk = self.lines[since:]
            if "<<done>>" in chunk:
                return "\n".join(chunk[:chunk.index("<<done>>")])
            if self.proc.poll() is not None:
                break
            time.sleep(0.02)
        raise TimeoutError(f"node {self.address}: command {line!r} did not finish:\n{self.output(since)}")

    def kill(self) -> None:
        if self.proc.poll() is None:
            os.killpg(self.proc.pid, signal.SIGKILL)
            self.proc.wait(timeout=10)

    def freeze(self) -> None:
        """A hung node (failure tests): SIGSTOP the process group. Its sockets
        stay open and nothing answers: peers see no FIN or RST, only silence.
        kill() still ends it."""
        if self.proc.poll() is None:
            os.killpg(self.proc.pid, signal.SIGSTOP)

    def stop(self) -> None:
        if self.proc.poll() is None:
            try:
                self.send("quit")
                self.proc.wait(timeout=5)
            except Exception:  # noqa: BLE001
                self.kill()


class LocalCluster:
    """N nodes on 127.0.0.1 at ports base, base+10, ...; the first
    ``n_leaders`` are leader candidates (in order)."""

    def __init__(self, n: int, base_port: int, root: str, labels: str, n_leaders: int = 2, **node_kw):
        self.root = root
        self.ports = [base_port + 10 * i for i in range(n)]
        self.leaders = [f"127.0.0.1:{p}" for p in self.ports[:n_leaders]]
        self.labels = labels
        self.node_kw = node_kw
        self.nodes: list[NodeProcess] = []

    def start(self, join: bool = True, timeout: float = 20.0) -> "LocalCluster":
        for p in self.ports:
            self.nodes.append(NodeProcess(p, self.leaders, os.path.join(self.root, f"n{p}"), self.labels,
                                          **self.node_kw))
        for nd in self.nodes:
            nd.expect(r"Address is", timeout)
        if join:
            intro = self.nodes[0].address
            for nd in self.nodes:
                nd.run(f"join {intro}", r"Joined!", timeout)
            self.wait_members(len(self.nodes), timeout)
        return self

    def wait_members(self, n: int, timeout: float = 20.0, nodes=None) -> None:
        deadline = time.time() + timeout
        for nd in nodes or self.nodes:
            if nd.proc.poll() is not None:
                continue
            while True:
                rows = len(re.findall(r"\| 127\.0\.0\.1:\d+ .*\| Active", nd.cmd("lm", 10)))
                if rows == n:
                    break
                if time.time() > deadline:
                    raise TimeoutError(f"{nd.address} sees {rows} active members, want {n}")
                time.sleep(0.2)

    def stop(self) -> None:
        for nd in self.nodes:
            nd.stop()
        for nd in self.nodes:
            nd.kill()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
