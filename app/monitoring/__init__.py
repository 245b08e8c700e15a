"""Monitoring / health service (port 9092)."""

from app.monitoring.service_monitor import MonitoringServer, ServiceMonitor

__all__ = ["ServiceMonitor", "MonitoringServer"]
