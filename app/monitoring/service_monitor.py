"""Monitoring server on port 9092 (API of the reference
``app/monitoring/service_monitor.py``: ``ServiceMonitor``, ``MonitoringServer``;
routes ``/health``, ``/health/ready``, ``/health/live``, ``/metrics``, ``/info``).

Changes: the WS server feeds the ``ServiceMonitor`` counters (Appendix D Q9);
``/metrics`` adds TTFT percentiles and, for the native provider, engine gauges
(running / waiting sequences, KV-cache usage, prefix-cache hit rate, step
latency) and per-GPU HBM use; ``/metrics/prometheus`` exposes the same numbers in
Prometheus text format; ``/health`` samples CPU without the reference's 1 s
blocking ``psutil.cpu_percent(interval=1)``.
"""
from __future__ import annotations

import logging
import threading
import time
from collections import deque
from typing import Any, Dict, Optional

import psutil

logger = logging.getLogger(__name__)


def _pct(xs, q):
    if not xs:
        return 0.0
    s = sorted(xs)
    i = min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))
    return s[i]


class ServiceMonitor:
    def __init__(self):
        self.start_time = time.time()
        self.request_count = 0
        self.generation_count = 0
        self.error_count = 0
        self.total_tokens_generated = 0
        self.total_processing_time = 0.0
        self._ttft = deque(maxlen=2048)
        self._lock = threading.Lock()
        self.server = None  # WebSocketLLMServer, for engine gauges
        self.node = None    # app.server.node_state.NodeBoard: DP workers feed this monitor

    def attach_server(self, server):
        self.server = server
        server.monitor = self

    def attach_node(self, board):
        """Parent of the DP service workers: /metrics sums the workers' counters
        (each worker publishes its own ServiceMonitor through the node board)."""
        self.node = board

    def counters(self) -> Dict[str, Any]:
        """Raw counters (published by a DP worker, summed by the parent)."""
        with self._lock:
            return {"requests": self.request_count, "generations": self.generation_count,
                    "errors": self.error_count, "total_tokens_generated": self.total_tokens_generated,
                    "total_processing_time": self.total_processing_time,
                    "ttft": list(self._ttft)[-256:]}

    def record_request(self):
        with self._lock:
            self.request_count += 1

    def record_generation(self, tokens: int, processing_time: float, ttft: Optional[float] = None):
        with self._lock:
            self.generation_count += 1
            self.total_tokens_generated += tokens
            self.total_processing_time += processing_time
            if ttft is not None:
                self._ttft.append(ttft)

    def record_error(self):
        with self._lock:
            self.error_count += 1

    def get_uptime(self) -> float:
        return time.time() - self.start_time

    def get_metrics(self) -> Dict[str, Any]:
        c = self.counters()
        snaps = []
        if self.node is not None:
            from app.server.node_state import merge_monitor

            snaps = [s for s in self.node.snapshots() if s]
            c = merge_monitor([c] + [s.get("monitor", {}) for s in snaps])
        n = c["generations"]
        m = {
            "uptime_seconds": self.get_uptime(),
            "requests": c["requests"],
            "generations": n,
            "errors": c["errors"],
            "total_tokens_generated": c["total_tokens_generated"],
            "avg_processing_time_seconds": c["total_processing_time"] / n if n else 0.0,
            "ttft_p50_ms": 1e3 * _pct(c["ttft"], 0.5),
            "ttft_p99_ms": 1e3 * _pct(c["ttft"], 0.99),
        }
        if self.node is not None:
            m["workers"] = self.node.workers()
            by = {s.get("index"): s for s in snaps}
            for w in m["workers"]:
                s = by.get(w["index"]) or {}
                w["generations"] = s.get("monitor", {}).get("generations", 0)
                if s.get("engine"):
                    w["engine"] = s["engine"]
        if self.server is not None:
            try:
                eng = self.server.engine_metrics()
                if eng:
                    m["engine"] = eng
            except Exception as e:  # pragma: no cover
                m["engine_error"] = str(e)
        gpu = _gpu_memory()
        if gpu:
            m["gpus"] = gpu
        return m


def _gpu_memory():
    try:
        import torch

        if not torch.cuda.is_available():
            return None
        out = []
        for i in range(torch.cuda.device_count()):
            free, total = torch.cuda.mem_get_info(i)
            out.append({"index": i, "hbm_used_gb": (total - free) / 2**30, "hbm_total_gb": total / 2**30})
        return out
    except Exception:
        return None


def prometheus_text(metrics: Dict[str, Any], prefix: str = "fasttalk") -> str:
    lines = []

    def emit(name, value, labels=""):
        if isinstance(value, bool):
            value = int(value)
        if isinstance(value, (int, float)):
            lines.append(f"{prefix}_{name}{labels} {value}")

    for k, v in metrics.items():
        if k == "engine" and isinstance(v, dict):
            for ek, ev in v.items():
                if isinstance(ev, dict):
                    for sk, sv in ev.items():
                        emit(f"engine_{ek}_{sk}", sv)
                else:
                    emit(f"engine_{ek}", ev)
        elif k == "workers" and isinstance(v, list):
            for w in v:
                lab = f'{{worker="{w["index"]}"}}'
                for wk in ("alive", "ready", "active_connections", "generations", "restarts"):
                    if wk in w:
                        emit(f"worker_{wk}", w[wk], lab)
        elif k == "gpus" and isinstance(v, list):
            for g in v:
                emit("gpu_hbm_used_gb", g["hbm_used_gb"], f'{{gpu="{g["index"]}"}}')
                emit("gpu_hbm_total_gb", g["hbm_total_gb"], f'{{gpu="{g["index"]}"}}')
        else:
            emit(k, v)
    return "\n".join(lines) + "\n"


class MonitoringServer:
    def __init__(self, host: str = "0.0.0.0", port: int = 9092, monitor: Optional[ServiceMonitor] = None):
        from flask import Flask

        self.host = host
        self.port = port
        self.monitor = monitor or ServiceMonitor()
        self.app = Flask(__name__)
        self._thread: Optional[threading.Thread] = None
        psutil.cpu_percent(interval=None)  # prime the non-blocking sampler
        self._register_routes()

    def _register_routes(self):
        from flask import Response, jsonify

        app = self.app

        @app.route("/health", methods=["GET"])
        def health():
            cpu = psutil.cpu_percent(interval=None)
            mem = psutil.virtual_memory()
            body = {
                "status": "healthy",
                "uptime_seconds": self.monitor.get_uptime(),
                "system": {"cpu_percent": cpu, "memory_percent": mem.percent,
                           "memory_available_gb": mem.available / 2**30},
                "metrics": self.monitor.get_metrics(),
            }
            warnings = []
            if cpu > 90:
                warnings.append("High CPU usage")
            if mem.percent > 90:
                warnings.append("High memory usage")
            if warnings:
                body["warnings"] = warnings
            return jsonify(body)

        @app.route("/health/ready", methods=["GET"])
        def ready():
            return jsonify({"status": "ready"})

        @app.route("/health/live", methods=["GET"])
        def live():
            return jsonify({"status": "live"})

        @app.route("/metrics", methods=["GET"])
        def metrics():
            return jsonify(self.monitor.get_metrics())

        @app.route("/metrics/prometheus", methods=["GET"])
        def metrics_prom():
            return Response(prometheus_text(self.monitor.get_metrics()), mimetype="text/plain")

        @app.route("/info", methods=["GET"])
        def info():
            return jsonify({"service": "llm-service", "version": "1.0.0",
                            "uptime_seconds": self.monitor.get_uptime()})

    def start(self):
        self._thread = threading.Thread(target=self._run_server, daemon=True, name="monitoring")
        self._thread.start()
        logger.info("Monitoring server started on %s:%s", self.host, self.port)

    def _run_server(self):
        from werkzeug.serving import make_server

        try:
            self._srv = make_server(self.host, self.port, self.app, threaded=True)
            self._srv.serve_forever()
        except OSError as e:
            logger.error("monitoring server failed: %s", e)

    def stop(self):
        srv = getattr(self, "_srv", None)
        if srv is not None:
            srv.shutdown()
