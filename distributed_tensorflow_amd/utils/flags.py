"""tf.app.flags-style flag definitions (reference trainer/task.py:17-31).

Flags are defined at import time and parsed lazily from ``sys.argv`` on first attribute access,
ignoring unknown flags — the behaviour the reference relies on when it calls ``main()`` directly
instead of ``tf.app.run``. Accepts ``--name=value``, ``--name value``, ``--flag``/
``--noflag`` for booleans.
"""
from __future__ import annotations

import sys


class _FlagValues:
    def __init__(self):
        object.__setattr__(self, "_defs", {})
        object.__setattr__(self, "_vals", {})
        object.__setattr__(self, "_parsed", False)

    def _define(self, name, default, help_, kind):
        self._defs[name] = (default, help_, kind)
        self._vals[name] = default

    def __call__(self, argv=None, known_only=True):
        argv = list(sys.argv[1:] if argv is None else argv)
        rest = []
        i = 0
        while i < len(argv):
            a = argv[i]
            if not a.startswith("--"):
                rest.append(a)
                i += 1
                continue
            body = a[2:]
            if "=" in body:
                k, v = body.split("=", 1)
            else:
                k, v = body, None
                if k not in self._defs and k.startswith("no") and k[2:] in self._defs and self._defs[k[2:]][2] is bool:
                    self._vals[k[2:]] = False
                    i += 1
                    continue
                if k in self._defs and self._defs[k][2] is not bool:
                    if i + 1 < len(argv):
                        v = argv[i + 1]
                        i += 1
            if k in self._defs:
                kind = self._defs[k][2]
                self._vals[k] = self._convert(kind, v)
            elif not known_only:
                raise ValueError(f"unknown flag --{k}")
            else:
                rest.append(a)
            i += 1
        object.__setattr__(self, "_parsed", True)
        return rest

    @staticmethod
    def _convert(kind, v):
        if kind is bool:
            return True if v is None else str(v).lower() in ("1", "true", "yes", "y", "t")
        if kind is list:
            return [] if not v else v.split(",")
        return kind(v)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        if not self._parsed:
            self(known_only=True)
        try:
            return self._vals[name]
        except KeyError:
            raise AttributeError(f"flag --{name} is not defined") from None

    def __setattr__(self, name, value):
        self._vals[name] = value

    def reset(self):
        for k, (d, _, _) in self._defs.items():
            self._vals[k] = d
        object.__setattr__(self, "_parsed", False)

    def flag_values_dict(self):
        if not self._parsed:
            self(known_only=True)
        return dict(self._vals)


FLAGS = _FlagValues()


def DEFINE_string(name, default, help_=""):
    FLAGS._define(name, default, help_, str)


def DEFINE_integer(name, default, help_=""):
    FLAGS._define(name, default, help_, int)


def DEFINE_float(name, default, help_=""):
    FLAGS._define(name, default, help_, float)


def DEFINE_boolean(name, default, help_=""):
    FLAGS._define(name, default, help_, bool)


DEFINE_bool = DEFINE_boolean


def DEFINE_list(name, default, help_=""):
    FLAGS._define(name, default, help_, list)
