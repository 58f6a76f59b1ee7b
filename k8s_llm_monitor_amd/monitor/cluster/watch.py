"""Resource and CRD watchers (``internal/k8s/watcher.go`` K3, ``crd_watcher.go`` K4).

``ResourceWatcher``: one thread per watched namespace x {pods, services, events}; each runs a
reconnect loop (5 s backoff after a stream ends or fails, watcher.go:74-87) and dispatches to an
``EventHandler`` (pods/services on ADDED/MODIFIED/DELETED, events on ADDED only).  Unlike the
reference it resumes from the last seen resourceVersion and re-lists on 410 Gone, and
``stop()`` is idempotent (the reference panics on a second ``close(stopCh)``).

``CRDWatcher``: watches CustomResourceDefinitions; starts a watcher per Established CRD (and on
ADDED), stops it on DELETED; keeps a cache of custom resources keyed ``group/kind/namespace`` and
emits ``CRDEvent``s.  Fixed vs the reference (Appendix A5 item 6): the CR watch carries the CRD's
storage version, a CR without ``spec`` does not crash, and the caches are lock-protected.
"""
from __future__ import annotations

import logging
import threading
from typing import Optional

from ...utils.gojson import utcnow
from ..types import CRDEvent, CRDInfo
from .backend import CRDS, EVENTS, GVR, PODS, SERVICES, ApiError, ClusterBackend
from .client import K8sClient, convert_custom_resource, convert_event, convert_pod, convert_service
from ...utils.gojson import parse_time, ZERO_TIME

log = logging.getLogger("k8s")


class EventHandler:
    """watcher.go:16-21."""

    def on_pod_update(self, pod) -> None: ...

    def on_service_update(self, svc) -> None: ...

    def on_event(self, ev) -> None: ...

    def on_crd_event(self, ev: CRDEvent) -> None: ...


class _Loop:
    def __init__(self, backend: ClusterBackend, gvr: GVR, namespace: Optional[str], on_event, stop: threading.Event,
                 backoff_s: float = 5.0, watch_timeout_s: float = 300.0):
        self.backend, self.gvr, self.namespace, self.on_event = backend, gvr, namespace, on_event
        self.stop, self.backoff_s, self.watch_timeout_s = stop, backoff_s, watch_timeout_s
        self.rv = ""
        self.thread = threading.Thread(target=self.run, daemon=True,
                                       name=f"watch-{gvr.resource}-{namespace or 'all'}")

    def run(self) -> None:
        while not self.stop.is_set():
            try:
                for etype, obj in self.backend.watch(self.gvr, self.namespace, self.rv, self.watch_timeout_s, self.stop):
                    if etype == "ERROR":
                        if obj.get("code") == 410:  # Gone: resourceVersion too old -> fresh watch
                            self.rv = ""
                        break
                    rv = obj.get("metadata", {}).get("resourceVersion")
                    if rv:
                        self.rv = rv
                    if etype == "BOOKMARK":
                        continue
                    try:
                        self.on_event(etype, obj)
                    except Exception as e:  # noqa: BLE001
                        log.warning("watch handler failed: %s", e)
                    if self.stop.is_set():
                        return
            except (ApiError, OSError) as e:
                log.error("Failed to watch %s in namespace %s: %s", self.gvr.resource, self.namespace, e)
            self.stop.wait(self.backoff_s)


class ResourceWatcher:
    def __init__(self, client: K8sClient, handler: EventHandler, backoff_s: float = 5.0,
                 watch_timeout_s: float = 300.0):
        self.client, self.handler = client, handler
        self._stop = threading.Event()
        self.loops: list[_Loop] = []
        self.backoff_s, self.watch_timeout_s = backoff_s, watch_timeout_s

    def start(self) -> None:
        log.info("Starting K8s resource watcher")
        for ns in self.client.namespaces:
            for gvr, fn in ((PODS, self._pod), (SERVICES, self._svc), (EVENTS, self._ev)):
                lp = _Loop(self.client.backend, gvr, ns, fn, self._stop, self.backoff_s, self.watch_timeout_s)
                self.loops.append(lp)
                lp.thread.start()

    def _pod(self, etype, obj):
        if etype in ("ADDED", "MODIFIED", "DELETED"):
            self.handler.on_pod_update(convert_pod(obj))

    def _svc(self, etype, obj):
        if etype in ("ADDED", "MODIFIED", "DELETED"):
            self.handler.on_service_update(convert_service(obj))

    def _ev(self, etype, obj):
        if etype == "ADDED":
            self.handler.on_event(convert_event(obj))

    def stop(self) -> None:
        if not self._stop.is_set():
            self._stop.set()
            log.info("K8s resource watcher stopped")


def convert_crd(crd: dict) -> CRDInfo:
    spec, st, md = crd.get("spec", {}), crd.get("status", {}), crd.get("metadata", {})
    return CRDInfo(name=md.get("name", ""), group=spec.get("group", ""), kind=spec.get("names", {}).get("kind", ""),
                   scope=spec.get("scope", ""), versions=[v.get("name", "") for v in spec.get("versions") or []],
                   plural=spec.get("names", {}).get("plural", ""), singular=spec.get("names", {}).get("singular", ""),
                   established=any(c.get("type") == "Established" and c.get("status") == "True"
                                   for c in st.get("conditions") or []),
                   stored=bool(st.get("storedVersions")),
                   creation_time=parse_time(md.get("creationTimestamp")) or ZERO_TIME)


def _storage_version(crd: dict) -> str:
    vs = crd.get("spec", {}).get("versions") or []
    for v in vs:
        if v.get("storage"):
            return v.get("name", "v1")
    return vs[0].get("name", "v1") if vs else "v1"


class CRDWatcher:
    def __init__(self, client: K8sClient, handler: Optional[EventHandler] = None, backoff_s: float = 5.0,
                 watch_timeout_s: float = 300.0):
        self.client, self.handler = client, handler
        self.backoff_s, self.watch_timeout_s = backoff_s, watch_timeout_s
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self.crds: dict[str, CRDInfo] = {}
        self.cr_stops: dict[str, threading.Event] = {}
        self.resources: dict[str, list] = {}

    def start(self) -> None:
        try:
            for crd in self.client.backend.list(CRDS):
                info = convert_crd(crd)
                if info.established:
                    self._start_cr(crd, info)
        except (ApiError, OSError) as e:
            log.warning("CRD discovery failed: %s", e)
        _Loop(self.client.backend, CRDS, None, self._on_crd, self._stop, self.backoff_s,
              self.watch_timeout_s).thread.start()

    def _on_crd(self, etype, crd):
        info = convert_crd(crd)
        if etype == "ADDED":
            self._start_cr(crd, info)
        elif etype == "DELETED":
            with self._lock:
                ev = self.cr_stops.pop(info.name, None)
                self.crds.pop(info.name, None)
            if ev:
                ev.set()

    def _start_cr(self, crd: dict, info: CRDInfo) -> None:
        with self._lock:
            if info.name in self.cr_stops:
                return
            stop = threading.Event()
            self.cr_stops[info.name] = stop
            self.crds[info.name] = info
        gvr = GVR(info.group, _storage_version(crd), info.plural, info.scope != "Cluster")
        both = _Either(self._stop, stop)

        def on_cr(etype, obj, info=info):
            cr = convert_custom_resource(obj, info.group, info.kind)
            key = f"{info.group}/{info.kind}/{cr.namespace}"
            with self._lock:
                lst = [r for r in self.resources.get(key, []) if r.name != cr.name]
                if etype in ("ADDED", "MODIFIED"):
                    lst.append(cr)
                self.resources[key] = lst
            if self.handler is not None:
                self.handler.on_crd_event(CRDEvent(type=etype, kind=info.kind, group=info.group, version=cr.version,
                                                   name=cr.name, namespace=cr.namespace, object=obj,
                                                   timestamp=utcnow()))

        _Loop(self.client.backend, gvr, None, on_cr, both, self.backoff_s, self.watch_timeout_s).thread.start()

    def get_crds(self) -> list:
        return [convert_crd(c) for c in self.client.backend.list(CRDS)]

    def get_custom_resources(self, group: str, kind: str, namespace: str) -> list:
        with self._lock:
            return list(self.resources.get(f"{group}/{kind}/{namespace}", []))

    def stop(self) -> None:
        self._stop.set()
        with self._lock:
            for ev in self.cr_stops.values():
                ev.set()


class _Either:
    """An Event view that is set when either of two events is set."""

    def __init__(self, a: threading.Event, b: threading.Event):
        self.a, self.b = a, b

    def is_set(self) -> bool:
        return self.a.is_set() or self.b.is_set()

    def wait(self, t: float) -> bool:
        import time as _t

        end = _t.monotonic() + t
        while _t.monotonic() < end:
            if self.is_set():
                return True
            _t.sleep(min(0.05, max(0.0, end - _t.monotonic())))
        return self.is_set()
