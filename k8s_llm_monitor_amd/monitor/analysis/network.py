"""Rule-based pod-communication diagnosis (K5) and the in-pod RTT tester (K6).

* ``NetworkAnalyzer.analyze_pod_communication`` = ``internal/k8s/network.go:34-82``: pod Running
  checks, NetworkPolicies of both namespaces (any-label match), a Service selecting pod B, CoreDNS
  Running, then the RTT test; final status ``connected``/0.9 or ``disconnected``/0.7
  (network.go:306-315).  Issue strings are the reference's, English for the static checks and
  Chinese for the RTT ones (Appendix A5 item 9, kept for API compatibility).
* ``RTTTester`` = ``internal/k8s/rtt_tester.go:43-369``: ``ping -c 3 -W 5`` both directions and
  ``curl -s -o /dev/null -w %{time_total} -m 5`` to HTTP-looking targets, run in the first
  container over pods/exec; output parsing and the latency grading (<1 ms excellent, <5 good,
  <50 fair, <100 poor).  Unlike the reference the whole test is bounded by a deadline so an
  analysis cannot outlive the 15 s HTTP write timeout (Appendix A5 item 11).
"""
from __future__ import annotations

import concurrent.futures as cf
import logging
import time
from typing import Optional

from ...utils.gojson import utcnow
from ..cluster.backend import NETWORK_POLICIES, PODS, ApiError
from ..cluster.client import K8sClient, convert_pod
from ..types import (CommunicationAnalysis, NetworkPolicyInfo, NetworkPolicyRule, NetworkTestResult, PodInfo,
                     PortRule, RTTResult)

log = logging.getLogger("k8s")


def parse_pod_name(ref: str) -> tuple[str, str]:
    """network.go:85-91: "ns/name" or bare "name" in "default"."""
    parts = ref.split("/")
    if len(parts) == 2:
        return parts[0], parts[1]
    return "default", parts[0]


def assess_latency(rtt: float) -> str:
    if rtt == 0:
        return "unknown"
    if rtt < 1:
        return "excellent"
    if rtt < 5:
        return "good"
    if rtt < 50:
        return "fair"
    if rtt < 100:
        return "poor"
    return "very_poor"


def parse_ping_output(output: str, r: RTTResult) -> None:
    """rtt_tester.go:219-250: mean of every ``time=X ms`` line; loss from the summary line."""
    total, n, loss = 0.0, 0, 0.0
    for line in output.splitlines():
        if "time=" in line and "ms" in line:
            part = line.split("time=", 1)[1].split(" ")[0]
            if part.endswith("ms"):
                part = part[:-2]
            try:
                v = float(part)
            except ValueError:
                v = 0.0
            if v > 0:
                total += v
                n += 1
        if "packet loss" in line:
            for tok in line.split(" "):
                if "%" in tok:
                    try:
                        loss = float(tok.rstrip("%"))
                        break
                    except ValueError:
                        continue
    if n > 0:
        r.rtt = total / n
        r.success = True
    r.packet_loss = loss


def parse_http_output(output: str, r: RTTResult) -> None:
    if not output:
        return
    try:
        v = float(output.strip())
    except ValueError:
        return
    r.rtt = v * 1000.0
    r.success = True
    r.packet_loss = 0.0


def is_http_service(pod: PodInfo) -> bool:
    app = (pod.labels or {}).get("app")
    if app is not None and any(h in app.lower() for h in ("nginx", "httpd", "apache", "web")):
        return True
    return any("nginx" in c.image.lower() or "httpd" in c.image.lower() for c in pod.containers or [])


class RTTTester:
    def __init__(self, client: K8sClient):
        self.client = client

    def _exec(self, namespace: str, pod: str, command: str, timeout_s: float) -> str:
        p = self.client.backend.get(PODS, pod, namespace)
        cs = p.get("spec", {}).get("containers") or []
        if not cs:
            raise RuntimeError(f"no containers found in pod {pod}")
        try:
            out, _ = self.client.backend.exec(namespace, pod, cs[0]["name"], ["sh", "-c", command], timeout_s)
        except Exception as e:  # noqa: BLE001
            raise RuntimeError(f"command execution failed: {e}") from e
        return out

    def _ping(self, src: PodInfo, ip: str, deadline: float) -> RTTResult:
        r = RTTResult(timestamp=utcnow(), success=False, method="ping")
        try:
            out = self._exec(src.namespace, src.name, f"ping -c 3 -W 5 {ip}", max(0.5, deadline - time.monotonic()))
        except Exception as e:  # noqa: BLE001
            r.error_message = f"执行ping命令失败: {e}"
            return r
        parse_ping_output(out, r)
        return r

    def _http(self, src: PodInfo, ip: str, port: int, deadline: float) -> RTTResult:
        r = RTTResult(timestamp=utcnow(), success=False, method="http")
        try:
            out = self._exec(src.namespace, src.name, f"curl -s -o /dev/null -w %{{time_total}} -m 5 http://{ip}:{port}",
                             max(0.5, deadline - time.monotonic()))
        except Exception as e:  # noqa: BLE001
            r.error_message = f"执行HTTP请求失败: {e}"
            return r
        parse_http_output(out, r)
        return r

    def test_pod_connectivity(self, pod_a: str, pod_b: str, timeout_s: float = 12.0) -> NetworkTestResult:
        deadline = time.monotonic() + timeout_s
        ans, an = parse_pod_name(pod_a)
        bns, bn = parse_pod_name(pod_b)
        try:
            a = convert_pod(self.client.backend.get(PODS, an, ans))
        except ApiError as e:
            raise RuntimeError(f"failed to get pod A info: {e}") from e
        try:
            b = convert_pod(self.client.backend.get(PODS, bn, bns))
        except ApiError as e:
            raise RuntimeError(f"failed to get pod B info: {e}") from e
        res = NetworkTestResult(pod_a=pod_a, pod_b=pod_b, rtt_results=[], test_count=0)
        # the three probes run concurrently (the reference runs them one after another)
        jobs = []
        with cf.ThreadPoolExecutor(max_workers=3) as ex:
            if b.ip:
                jobs.append(("ping", ex.submit(self._ping, a, b.ip, deadline)))
            if a.ip:
                jobs.append(("ping_reverse", ex.submit(self._ping, b, a.ip, deadline)))
            if is_http_service(b):
                jobs.append(("http", ex.submit(self._http, a, b.ip, 80, deadline)))
            for method, f in jobs:
                try:
                    r = f.result(timeout=max(0.1, deadline - time.monotonic()))
                except cf.TimeoutError:
                    r = RTTResult(timestamp=utcnow(), success=False, error_message="test timed out")
                r.method = method
                res.rtt_results.append(r)
                res.test_count += 1
        ok = [r for r in res.rtt_results if r.success]
        if res.rtt_results:
            res.average_rtt = sum(r.rtt for r in ok) / len(ok) if ok else 0.0
            res.success_rate = len(ok) / len(res.rtt_results) * 100 if ok else 0.0
            res.latency = assess_latency(res.average_rtt)
        else:
            res.average_rtt, res.success_rate, res.latency = 0.0, 0.0, "unknown"
        return res


def convert_network_policy(np_: dict) -> NetworkPolicyInfo:
    """network.go:149-181 (without its nil dereference on port rules lacking protocol/port)."""
    md, spec = np_.get("metadata", {}), np_.get("spec", {})

    def rules(key):
        out = None
        for rule in spec.get(key) or []:
            pr = None
            for p in rule.get("ports") or []:
                port = p.get("port")
                (pr := pr or []).append(PortRule(protocol=p.get("protocol") or "TCP",
                                                 port=port if isinstance(port, int) else 0))
            (out := out or []).append(NetworkPolicyRule(ports=pr))
        return out

    return NetworkPolicyInfo(name=md.get("name", ""), namespace=md.get("namespace", ""),
                             pod_selector=(spec.get("podSelector") or {}).get("matchLabels") or None,
                             ingress=rules("ingress"), egress=rules("egress"))


def _any_label_match(selector: Optional[dict], labels: Optional[dict]) -> bool:
    """The reference's OR-semantics (network.go:199-208,237-244; Appendix A5 item 5): any single
    matching label counts, and an empty selector never matches."""
    labels = labels or {}
    return any(labels.get(k) == v for k, v in (selector or {}).items())


class NetworkAnalyzer:
    def __init__(self, client: K8sClient, enable_rtt: bool = True, rtt_timeout_s: float = 10.0):
        self.client = client
        self.rtt = RTTTester(client)
        self.enable_rtt = enable_rtt
        self.rtt_timeout_s = rtt_timeout_s
        self.last_rtt: Optional[NetworkTestResult] = None

    def analyze_pod_communication(self, pod_a: str, pod_b: str) -> CommunicationAnalysis:
        ans, an = parse_pod_name(pod_a)
        bns, bn = parse_pod_name(pod_b)
        try:
            a = self.client.get_pod(ans, an)
        except ApiError as e:
            raise RuntimeError(f"failed to get pod A info: {e}") from e
        try:
            b = self.client.get_pod(bns, bn)
        except ApiError as e:
            raise RuntimeError(f"failed to get pod B info: {e}") from e
        an_ = CommunicationAnalysis(pod_a=pod_a, pod_b=pod_b, status="unknown", issues=[], solutions=[],
                                    confidence=0.0)
        for p in (a, b):
            if p.status != "Running":
                an_.issues.append(f"Pod {p.namespace}/{p.name} is not running (status: {p.status})")
                an_.solutions.append(f"Check Pod {p.namespace}/{p.name} logs and events for issues")
        self._check_policies(a, b, an_)
        self._check_service(b, an_)
        self._check_dns(an_)
        if self.enable_rtt:
            self._check_rtt(pod_a, pod_b, an_)
        if not an_.issues:
            an_.status, an_.confidence = "connected", 0.9
            an_.solutions.append("No obvious issues detected")
        else:
            an_.status, an_.confidence = "disconnected", 0.7
        return an_

    def _check_policies(self, a: PodInfo, b: PodInfo, an_: CommunicationAnalysis) -> None:
        pols = []
        for ns in (a.namespace, b.namespace):
            try:
                pols += [convert_network_policy(p) for p in self.client.backend.list(NETWORK_POLICIES, ns)]
            except (ApiError, OSError) as e:
                log.warning("Failed to get network policies for namespace %s: %s", ns, e)
                return
        for pol in pols:
            if _any_label_match(pol.pod_selector, a.labels) or _any_label_match(pol.pod_selector, b.labels):
                an_.issues.append(f"Network policy {pol.namespace}/{pol.name} may affect communication")
                an_.solutions.append(f"Review network policy {pol.namespace}/{pol.name} rules")

    def _check_service(self, b: PodInfo, an_: CommunicationAnalysis) -> None:
        try:
            svcs = self.client.get_services(b.namespace) or []
        except (ApiError, OSError) as e:
            log.warning("Failed to get services for namespace %s: %s", b.namespace, e)
            return
        if not any(_any_label_match(s.selector, b.labels) for s in svcs):
            an_.issues.append(f"No service found targeting Pod {b.namespace}/{b.name}")
            an_.solutions.append(f"Create a service to expose Pod {b.namespace}/{b.name}")

    def _check_dns(self, an_: CommunicationAnalysis) -> None:
        try:
            pods = self.client.get_pods("kube-system") or []
        except (ApiError, OSError) as e:
            log.warning("Failed to get CoreDNS pods: %s", e)
            return
        if not any("coredns" in p.name and p.status == "Running" for p in pods):
            an_.issues.append("CoreDNS is not running properly")
            an_.solutions.append("Check CoreDNS pods in kube-system namespace")

    def _check_rtt(self, pod_a: str, pod_b: str, an_: CommunicationAnalysis) -> None:
        try:
            r = self.rtt.test_pod_connectivity(pod_a, pod_b, timeout_s=self.rtt_timeout_s)
        except Exception as e:  # noqa: BLE001
            an_.issues.append(f"RTT测试失败: {e}")
            an_.solutions.append("检查Pod是否支持网络命令执行")
            return
        self.last_rtt = r
        if r.success_rate < 50:
            an_.issues.append(f"网络连通性差，成功率仅为{r.success_rate:.1f}%")
            an_.solutions.append("检查网络策略和防火墙配置")
        elif r.success_rate < 100:
            an_.issues.append(f"网络存在丢包，成功率为{r.success_rate:.1f}%")
            an_.solutions.append("检查网络质量和节点状态")
        if r.latency == "fair":
            an_.issues.append(f"网络延迟一般，平均RTT为{r.average_rtt:.2f}ms")
            an_.solutions.append("考虑优化网络配置或检查网络负载")
        elif r.latency in ("poor", "very_poor"):
            an_.issues.append(f"网络延迟较高，平均RTT为{r.average_rtt:.2f}ms")
            an_.solutions.append("检查网络配置和节点间网络连接")
