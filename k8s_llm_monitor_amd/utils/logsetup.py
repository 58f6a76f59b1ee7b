"""``logging.*`` config honoured (level / format json|text / output stdout|stderr|<file>) - the
reference declares these keys but ignores them."""
from __future__ import annotations

import json
import logging
import sys
import time


class JSONFormatter(logging.Formatter):
    def format(self, r: logging.LogRecord) -> str:
        d = {"time": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(r.created)) + f".{int(r.msecs):03d}Z",
             "level": r.levelname.lower(), "logger": r.name, "msg": r.getMessage()}
        if r.exc_info:
            d["error"] = self.formatException(r.exc_info)
        return json.dumps(d, ensure_ascii=False)


def setup_logging(level: str = "info", fmt: str = "json", output: str = "stdout") -> None:
    root = logging.getLogger()
    for h in list(root.handlers):
        root.removeHandler(h)
    if output in ("", "stdout"):
        h = logging.StreamHandler(sys.stdout)
    elif output == "stderr":
        h = logging.StreamHandler(sys.stderr)
    else:
        h = logging.FileHandler(output)
    h.setFormatter(JSONFormatter() if fmt == "json" else
                   logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
    root.addHandler(h)
    root.setLevel({"debug": logging.DEBUG, "info": logging.INFO, "warn": logging.WARNING, "warning": logging.WARNING,
                   "error": logging.ERROR, "fatal": logging.CRITICAL}.get((level or "info").lower(), logging.INFO))
