"""shadow.yaml front end: the reference's configuration API for the packet core, restated.

What the reference does (src/main/shadow.rs:96-100, core/configuration.rs, core/sim_config.rs)
and what this module mirrors, step by step:

1. load_config_file (shadow.rs:370-407): serde_yaml parses the file into a YAML Value
   (duplicate keys are an error), applies '<<' merge keys and drops top-level 'x-*' keys
   (extended YAML is always on, shadow.rs:96), then deserializes ConfigFileOptions with
   deny_unknown_fields on every struct (configuration.rs:92-109).  YAML scalars resolve as
   serde_yaml 0.9 does (YAML 1.2 core schema: 'off'/'yes' are strings, '010' is a string).
2. ConfigOptions::new (configuration.rs:124-154): host_option_defaults merged with the real
   defaults, command-line options override the file (clap flags = kebab-case field names),
   the merged host defaults are copied into every host.
3. SimConfig::new (sim_config.rs:47-164): hosts in hostname order (BTreeMap), per-host seeds
   (sgn_derive_host_seeds), the graph (gml inline / file / xz / 1_gbit_switch,
   graph/mod.rs:478-507) through sgn_gml_parse, node-id checks, bandwidths (incl. the
   bandwidth_up <- bandwidth_down quirk, sim_config.rs:249-254), IP assignment through
   sgn_assign_ips (sim_config.rs:386-407), used nodes = nodes with a host.

Process/plugin resolution (which::which, sim_config.rs:335-368) is out of scope (SURVEY.md
§2 row 9): process entries are validated and kept, never executed.  Synthetic traffic is not
part of shadow.yaml (unknown keys are rejected) and comes from the caller (bench.py / tests).
Everything numeric of the packet core runs in libsgn; this module only shapes its inputs.
"""
from __future__ import annotations

import copy
import ipaddress
import lzma
import os
import re
from dataclasses import dataclass, field

import numpy as np
import yaml

import sgn


class ConfigError(ValueError):
    """A configuration the reference rejects (the message names the offending field)."""


# --------------------------------------------------------------------------------------
# YAML with serde_yaml 0.9 scalar resolution
# --------------------------------------------------------------------------------------

_FLOAT = re.compile(r"^[-]?(?:[0-9]+\.?[0-9]*|\.[0-9]+)(?:[eE][+-]?[0-9]+)?$")


def _digits_but_not_number(s):
    t = s[1:] if s[:1] in "+-" else s
    return len(t) > 1 and t[0] == "0" and t[1:].isdigit() and t.isascii()


def _parse_int(s):
    """serde_yaml parse_unsigned_int / parse_negative_int: 0x/0o/0b prefixes, decimal
    without leading zeros, at most one sign."""
    neg = s.startswith("-")
    body = s[1:] if s[:1] in "+-" else s
    for pfx, radix in (("0x", 16), ("0o", 8), ("0b", 2)):
        if body.startswith(pfx):
            rest = body[2:]
            if rest and rest[:1] not in "+-_" and re.fullmatch(r"[0-9a-fA-F]+", rest):
                try:
                    v = int(rest, radix)
                    return -v if neg else v
                except ValueError:
                    return None
            return None
    if body[:1] in "+-" or not body.isascii() or not body.isdigit() or _digits_but_not_number(s):
        return None
    v = int(body)
    return -v if neg else v


def _resolve_plain(s):
    if s in ("", "~", "null", "Null", "NULL"):
        return None
    if s in ("true", "True", "TRUE"):
        return True
    if s in ("false", "False", "FALSE"):
        return False
    v = _parse_int(s)
    if v is not None and -(1 << 127) <= v < (1 << 128):
        return v
    if not _digits_but_not_number(s):
        u = s[1:] if s.startswith("+") else s
        if u in (".inf", ".Inf", ".INF"):
            return float("inf")
        if s in ("-.inf", "-.Inf", "-.INF"):
            return float("-inf")
        if s in (".nan", ".NaN", ".NAN"):
            return float("nan")
        if not u.startswith(("+",)) and _FLOAT.match(u):
            f = float(u)
            if f == f and abs(f) != float("inf"):
                return f
    return s


class _Loader(yaml.SafeLoader):
    """Composes nodes with PyYAML, resolves scalars and mappings like serde_yaml::Value."""


_Loader.yaml_implicit_resolvers = {}  # no YAML 1.1 implicit typing: every plain scalar -> str


def _construct_plain_or_str(loader, node):
    v = loader.construct_scalar(node)
    return _resolve_plain(v) if node.style is None else v


def _construct_mapping(loader, node):
    out = {}
    for k_node, v_node in node.value:
        k = loader.construct_object(k_node, deep=True)
        if isinstance(k, (dict, list)):
            raise ConfigError("Could not parse configuration file as yaml: non-scalar mapping key")
        if (type(k), k) in {(type(x), x) for x in out}:
            raise ConfigError(f"Could not parse configuration file as yaml: duplicate entry with key \"{k}\"")
        out[k] = loader.construct_object(v_node, deep=True)
    return out


def _construct_seq(loader, node):
    return [loader.construct_object(n, deep=True) for n in node.value]


_Loader.yaml_constructors = dict(yaml.SafeLoader.yaml_constructors)
_Loader.add_constructor("tag:yaml.org,2002:str", _construct_plain_or_str)
_Loader.add_constructor("tag:yaml.org,2002:map", _construct_mapping)
_Loader.add_constructor("tag:yaml.org,2002:seq", _construct_seq)


def _apply_merge(root):
    """serde_yaml::Value::apply_merge: '<<: mapping' or '<<: [mappings]' fill keys the
    mapping does not have; merged-in values are themselves processed."""
    stack = [root]
    while stack:
        node = stack.pop()
        if isinstance(node, dict):
            if "<<" in node:
                m = node.pop("<<")
                if isinstance(m, dict):
                    srcs = [m]
                elif isinstance(m, list):
                    for x in m:
                        if isinstance(x, list):
                            raise ConfigError("Could not merge '<<' keys: expected a mapping for merging, but found sequence")
                        if not isinstance(x, dict):
                            raise ConfigError("Could not merge '<<' keys: expected a mapping for merging, but found scalar")
                    srcs = m
                else:
                    raise ConfigError("Could not merge '<<' keys: expected a mapping or list of mappings for merging, but found scalar")
                for s in srcs:
                    for k, v in s.items():
                        if k not in node:
                            node[k] = v
            stack.extend(node.values())
        elif isinstance(node, list):
            stack.extend(node)


def load_yaml(text):
    """load_config_file (shadow.rs:370-407) up to serde_yaml::from_value."""
    try:
        doc = yaml.load(text, Loader=_Loader)  # noqa: S506 - safe loader subclass, no tags
    except yaml.YAMLError as e:
        raise ConfigError(f"Could not parse configuration file as yaml: {e}") from None
    doc = copy.deepcopy(doc)  # aliases become independent copies, as in serde_yaml::Value
    _apply_merge(doc)
    if isinstance(doc, dict):
        for k in [k for k in doc if isinstance(k, str) and k.startswith("x-")]:
            del doc[k]
    return doc


# --------------------------------------------------------------------------------------
# Units (utility/units.rs): value + prefix, Display, checked conversion to the base unit
# --------------------------------------------------------------------------------------

_TIME = {"ns": ("ns", 1), "nanosecond": ("ns", 1), "nanoseconds": ("ns", 1),
         "us": ("μs", 10**3), "μs": ("μs", 10**3), "microsecond": ("μs", 10**3),
         "microseconds": ("μs", 10**3),
         "ms": ("ms", 10**6), "millisecond": ("ms", 10**6), "milliseconds": ("ms", 10**6),
         "s": ("sec", 10**9), "sec": ("sec", 10**9), "secs": ("sec", 10**9),
         "second": ("sec", 10**9), "seconds": ("sec", 10**9),
         "m": ("min", 60 * 10**9), "min": ("min", 60 * 10**9), "mins": ("min", 60 * 10**9),
         "minute": ("min", 60 * 10**9), "minutes": ("min", 60 * 10**9),
         "h": ("hour", 3600 * 10**9), "hr": ("hour", 3600 * 10**9), "hrs": ("hour", 3600 * 10**9),
         "hour": ("hour", 3600 * 10**9), "hours": ("hour", 3600 * 10**9)}
_SI_UPPER = {"K": ("K", 10**3), "kilo": ("K", 10**3), "Ki": ("Ki", 2**10), "kibi": ("Ki", 2**10),
             "M": ("M", 10**6), "mega": ("M", 10**6), "Mi": ("Mi", 2**20), "mebi": ("Mi", 2**20),
             "G": ("G", 10**9), "giga": ("G", 10**9), "Gi": ("Gi", 2**30), "gibi": ("Gi", 2**30),
             "T": ("T", 10**12), "tera": ("T", 10**12), "Ti": ("Ti", 2**40), "tebi": ("Ti", 2**40)}
_UNIT_KINDS = {
    # kind: (suffixes, prefix table, default prefix (display, factor))
    "time": ([""], _TIME, ("sec", 10**9)),
    "bytes": (["B", "byte", "bytes"], _SI_UPPER, ("", 1)),
    "bits": (["bit", "bits"], _SI_UPPER, ("", 1)),
}
_U64 = (1 << 64) - 1
# Rust's \s: Unicode White_Space
_WS = "\t\n\x0b\x0c\r \x85\xa0                　"


@dataclass(frozen=True)
class Unit:
    kind: str
    value: int
    prefix: str  # display form: "sec", "μs", "G", ""
    factor: int  # base units per 1 of this prefix

    def base(self) -> int:
        """convert(base prefix) with checked_mul (units.rs:378-389)."""
        v = self.value * self.factor
        if v > _U64:
            raise ConfigError(f"The resulting value is outside of the bounds [0, {_U64}]")
        return v

    def __str__(self):
        return f"{self.value} {self.prefix}{_UNIT_KINDS[self.kind][0][0]}"

    @classmethod
    def parse(cls, kind, s):
        """FromStr (units.rs:406-440): ^([+-]?[0-9\\.]*)\\s*(.*)$, value.trim() as u64."""
        suffixes, table, default = _UNIT_KINDS[kind]
        m = re.match(r"^([+-]?[0-9.]*)[" + _WS + r"]*([^\n]*)$", s)
        if not m:
            raise ConfigError(f"invalid {kind} value {s!r}: Unable to identify value and unit")
        num, unit = m.group(1).strip(_WS), m.group(2).strip(_WS)
        prefix = unit
        for sfx in suffixes:
            if unit.endswith(sfx):
                prefix = unit[: len(unit) - len(sfx)]
                break
        if prefix == "":
            disp, factor = default
        elif prefix in table:
            disp, factor = table[prefix]
        else:
            raise ConfigError(f"invalid {kind} value {s!r}: unknown unit prefix {prefix!r}")
        body = num[1:] if num.startswith("+") else num
        if not body or not body.isdigit() or int(body) > _U64:
            raise ConfigError(f"invalid {kind} value {s!r}: invalid digit found in string")
        return cls(kind, int(body), disp, factor)

    @classmethod
    def from_yaml(cls, kind, v, where):
        if isinstance(v, bool) or v is None:
            raise ConfigError(f"{where}: invalid type, expected a {kind} value")
        if isinstance(v, int):  # visit_u64/i64: value with the default prefix
            if v < 0 or v > _U64:
                raise ConfigError(f"{where}: out of range integral type conversion attempted")
            disp, factor = _UNIT_KINDS[kind][2]
            return cls(kind, v, disp, factor)
        if isinstance(v, str):
            try:
                return cls.parse(kind, v)
            except ConfigError as e:
                raise ConfigError(f"{where}: {e}") from None
        raise ConfigError(f"{where}: invalid type: {type(v).__name__}, expected struct {kind}")


# --------------------------------------------------------------------------------------
# Schema (configuration.rs): field -> (parser, serde default)
# --------------------------------------------------------------------------------------

NULL = "null"  # NullableOption::Null (only the command line can produce it)
_MISSING = object()

SIGNALS = {"SIGHUP": 1, "SIGINT": 2, "SIGQUIT": 3, "SIGILL": 4, "SIGTRAP": 5, "SIGABRT": 6,
           "SIGBUS": 7, "SIGFPE": 8, "SIGKILL": 9, "SIGUSR1": 10, "SIGSEGV": 11, "SIGUSR2": 12,
           "SIGPIPE": 13, "SIGALRM": 14, "SIGTERM": 15, "SIGSTKFLT": 16, "SIGCHLD": 17,
           "SIGCONT": 18, "SIGSTOP": 19, "SIGTSTP": 20, "SIGTTIN": 21, "SIGTTOU": 22,
           "SIGURG": 23, "SIGXCPU": 24, "SIGXFSZ": 25, "SIGVTALRM": 26, "SIGPROF": 27,
           "SIGWINCH": 28, "SIGIO": 29, "SIGPWR": 30, "SIGSYS": 31}
_SIGNAL_NAMES = {v: k for k, v in SIGNALS.items()}


class _Field:
    """A field type: .yaml() deserializes a YAML value, .cli() is clap's FromStr."""

    def cli(self, text, where):
        return self.yaml(text, where)


class _Bool(_Field):
    def yaml(self, v, where):
        if not isinstance(v, bool):
            raise ConfigError(f"{where}: invalid type: expected a boolean")
        return v

    def cli(self, text, where):
        if text not in ("true", "false"):
            raise ConfigError(f"{where}: invalid value '{text}' for bool")
        return text == "true"


class _U32(_Field):
    def yaml(self, v, where):
        if isinstance(v, bool) or not isinstance(v, int):
            raise ConfigError(f"{where}: invalid type: expected u32")
        if not 0 <= v <= 0xFFFFFFFF:
            raise ConfigError(f"{where}: invalid value: integer `{v}`, expected u32")
        return v

    def cli(self, text, where):
        if not re.fullmatch(r"\+?[0-9]+", text):
            raise ConfigError(f"{where}: invalid digit found in string")
        return self.yaml(int(text), where)


class _Str(_Field):
    def yaml(self, v, where):
        if not isinstance(v, str):
            raise ConfigError(f"{where}: invalid type: expected a string")
        return v


class _Enum(_Field):
    def __init__(self, *names):
        self.names = names

    def yaml(self, v, where):
        if not isinstance(v, str) or v not in self.names:
            raise ConfigError(f"{where}: unknown variant `{v}`, expected one of {', '.join(self.names)}")
        return v


class _UnitF(_Field):
    def __init__(self, kind):
        self.kind = kind

    def yaml(self, v, where):
        return Unit.from_yaml(self.kind, v, where)

    def cli(self, text, where):
        try:
            return Unit.parse(self.kind, text)
        except ConfigError as e:
            raise ConfigError(f"{where}: {e}") from None


_p_bool, _p_u32, _p_str = _Bool().yaml, _U32().yaml, _Str().yaml
_BOOL, _U32_, _STR = _Bool(), _U32(), _Str()
_TIME_F, _BYTES_F = _UnitF("time"), _UnitF("bytes")


def _p_signal(v, where):
    if isinstance(v, str):
        if v not in SIGNALS:
            raise ConfigError(f"{where}: Invalid signal string: {v}")
        return v
    if isinstance(v, int) and not isinstance(v, bool):
        if v not in _SIGNAL_NAMES:
            raise ConfigError(f"{where}: Invalid signal number: {v}")
        return _SIGNAL_NAMES[v]
    raise ConfigError(f"{where}: invalid type: expected a signal string (e.g. \"SIGINT\") or integer")


_LOG_LEVEL = _Enum("error", "warning", "info", "debug", "trace")

# (name, parser, serde default, nullable-on-CLI)  -- configuration.rs:222-296
GENERAL = [
    ("stop_time", _TIME_F, None, False),
    ("seed", _U32_, 1, False),
    ("parallelism", _U32_, 0, False),
    ("bootstrap_end_time", _TIME_F, Unit("time", 0, "sec", 10**9), False),
    ("log_level", _LOG_LEVEL, "info", False),
    ("heartbeat_interval", _TIME_F, Unit("time", 1, "sec", 10**9), True),
    ("data_directory", _STR, "shadow.data", False),
    ("template_directory", _STR, None, True),
    ("progress", _BOOL, False, False),
    ("model_unblocked_syscall_latency", _BOOL, False, False),
]
# configuration.rs:310-327; graph is not a CLI option (clap(skip))
NETWORK = [
    ("graph", None, None, False),
    ("use_shortest_path", _BOOL, True, False),
]
_T = lambda v, p, f: Unit("time", v, p, f)  # noqa: E731
# configuration.rs:345-581 (ExperimentalOptions::default)
EXPERIMENTAL = [
    ("use_sched_fifo", _BOOL, False, False),
    ("use_syscall_counters", _BOOL, True, False),
    ("use_object_counters", _BOOL, True, False),
    ("use_preload_libc", _BOOL, True, False),
    ("use_preload_openssl_rng", _BOOL, True, False),
    ("use_preload_openssl_crypto", _BOOL, False, False),
    ("use_memory_manager", _BOOL, False, False),
    ("use_cpu_pinning", _BOOL, True, False),
    ("use_worker_spinning", _BOOL, True, False),
    ("runahead", _TIME_F, _T(1, "ms", 10**6), True),
    ("use_dynamic_runahead", _BOOL, False, False),
    ("socket_send_buffer", _BYTES_F, Unit("bytes", 131_072, "", 1), False),
    ("socket_send_autotune", _BOOL, True, False),
    ("socket_recv_buffer", _BYTES_F, Unit("bytes", 174_760, "", 1), False),
    ("socket_recv_autotune", _BOOL, True, False),
    ("interface_qdisc", _Enum("fifo", "round-robin"), "fifo", False),
    ("strace_logging_mode", _Enum("off", "standard", "deterministic"), "off", False),
    ("max_unapplied_cpu_latency", _TIME_F, _T(1, "μs", 10**3), False),
    ("unblocked_syscall_latency", _TIME_F, _T(1, "μs", 10**3), False),
    ("unblocked_vdso_latency", _TIME_F, _T(10, "ns", 1), False),
    ("scheduler", _Enum("thread-per-host", "thread-per-core"), "thread-per-core", False),
    ("report_errors_to_stderr", _BOOL, True, False),
    ("use_new_tcp", _BOOL, False, False),
    ("native_preemption_enabled", _BOOL, False, False),
    ("native_preemption_native_interval", _TIME_F, _T(100, "ms", 10**6), False),
    ("native_preemption_sim_interval", _TIME_F, _T(10, "ms", 10**6), False),
]
# configuration.rs:591-623 (HostDefaultOptions; new_with_defaults supplies the defaults)
HOST_DEFAULTS = [
    ("log_level", _LOG_LEVEL, None, True),
    ("pcap_enabled", _BOOL, False, False),
    ("pcap_capture_size", _BYTES_F, Unit("bytes", 65535, "", 1), False),
]
# CLI long names that differ from the kebab-case field name, and short flags
_CLI_RENAME = {("host_option_defaults", "log_level"): "host-log-level"}
_CLI_SHORT = {"p": ("general", "parallelism"), "l": ("general", "log_level"),
              "d": ("general", "data_directory"), "e": ("general", "template_directory")}


def _where(path, k=None):
    return ".".join([*path, str(k)] if k is not None else path) or "<root>"


def _check_keys(m, allowed, path):
    if not isinstance(m, dict):
        raise ConfigError(f"{_where(path)}: invalid type: expected a mapping")
    for k in m:
        if k not in allowed:
            raise ConfigError(f"{_where(path)}: unknown field `{k}`, expected one of "
                              + ", ".join(f"`{a}`" for a in allowed))


def _section(m, schema, path, struct_default):
    """A deny_unknown_fields struct of Option fields. struct_default=True: a missing field
    takes the schema default (serde(default) on the struct or on the field); YAML null is
    None (unset) either way."""
    _check_keys(m, [f[0] for f in schema], path)
    out = {}
    for name, parse, default, _ in schema:
        if name in m:
            v = m[name]
            out[name] = None if v is None else (parse.yaml(v, _where(path, name)) if parse else v)
        else:
            out[name] = default if struct_default else None
    return out


def _graph(v, where):
    """GraphOptions (configuration.rs:985-1015): internally tagged by `type`."""
    if not isinstance(v, dict) or "type" not in v:
        raise ConfigError(f"{where}: missing field `type`")
    t = v["type"]
    rest = {k: x for k, x in v.items() if k != "type"}
    if t == "1_gbit_switch":
        return {"type": "1_gbit_switch"}
    if t != "gml":
        raise ConfigError(f"{where}: unknown variant `{t}`, expected `gml` or `1_gbit_switch`")
    if len(rest) != 1:
        raise ConfigError(f"{where}: expected exactly one of `file`, `inline`")
    (k, x), = rest.items()
    if k == "inline":
        return {"type": "gml", "inline": _p_str(x, f"{where}.inline")}
    if k == "file":
        _check_keys(x, ["path", "compression"], [where, "file"])
        if "path" not in x:
            raise ConfigError(f"{where}.file: missing field `path`")
        comp = x.get("compression")
        if comp is not None and comp != "xz":
            raise ConfigError(f"{where}.file.compression: unknown variant `{comp}`, expected `xz`")
        return {"type": "gml", "file": {"path": _p_str(x["path"], f"{where}.file.path"),
                                        "compression": comp}}
    raise ConfigError(f"{where}: unknown variant `{k}`, expected `file` or `inline`")


def _hostname(k):
    """HostName (configuration.rs:786-842)."""
    if not isinstance(k, str):
        raise ConfigError("hosts: invalid type: expected a string hostname")
    bad = next((c for c in k if not (("a" <= c <= "z") or ("0" <= c <= "9") or c in "-.")), None)
    if bad is not None:
        raise ConfigError(f"hosts: invalid hostname character: '{bad}'")
    if not k:
        raise ConfigError("hosts: empty hostname")
    if k.startswith("-"):
        raise ConfigError("hosts: hostname begins with a '-' character")
    if len(k) > 253:
        raise ConfigError("hosts: hostname exceeds 253 characters")
    return k


def _process(p, where):
    """ProcessOptions (configuration.rs:627-652)."""
    fields = ["path", "args", "environment", "start_time", "shutdown_time", "shutdown_signal",
              "expected_final_state"]
    _check_keys(p, fields, [where])
    if "path" not in p:
        raise ConfigError(f"{where}: missing field `path`")
    args = p.get("args", "")
    if isinstance(args, list):
        args = [_p_str(a, f"{where}.args") for a in args]
    elif not isinstance(args, str):
        raise ConfigError(f"{where}.args: invalid type: expected a string or a sequence of strings")
    env = p.get("environment", {})
    if env is None:
        env = {}
    if not isinstance(env, dict):
        raise ConfigError(f"{where}.environment: invalid type: expected a map")
    for k, x in env.items():
        if not isinstance(k, str) or "=" in k:
            raise ConfigError(f"{where}.environment: environment variable name contains a '=' character")
        _p_str(x, f"{where}.environment.{k}")
    efs = p.get("expected_final_state", {"exited": 0})
    if efs == "running":
        pass
    elif isinstance(efs, dict) and "exited" in efs:
        v = efs["exited"]
        if isinstance(v, bool) or not isinstance(v, int) or not -(1 << 31) <= v < (1 << 31):
            raise ConfigError(f"{where}.expected_final_state: invalid exit code")
        efs = {"exited": v}
    elif isinstance(efs, dict) and "signaled" in efs:
        efs = {"signaled": _p_signal(efs["signaled"], f"{where}.expected_final_state.signaled")}
    else:
        raise ConfigError(f"{where}.expected_final_state: data did not match any variant")
    st = p.get("start_time")
    sh = p.get("shutdown_time")
    return {
        "path": _p_str(p["path"], f"{where}.path"),
        "args": args,
        "environment": dict(sorted(env.items())),
        "start_time": Unit("time", 0, "sec", 10**9) if st is None else Unit.from_yaml("time", st, f"{where}.start_time"),
        "shutdown_time": None if sh is None else Unit.from_yaml("time", sh, f"{where}.shutdown_time"),
        "shutdown_signal": "SIGTERM" if p.get("shutdown_signal") is None else _p_signal(p["shutdown_signal"], f"{where}.shutdown_signal"),
        "expected_final_state": efs,
    }


def _ipv4(v, where):
    """std::net::Ipv4Addr FromStr: four decimal octets, no leading zeros."""
    if not isinstance(v, str) or not re.fullmatch(r"(0|[1-9][0-9]{0,2})(\.(0|[1-9][0-9]{0,2})){3}", v) \
            or any(int(o) > 255 for o in v.split(".")):
        raise ConfigError(f"{where}: invalid IP address syntax")
    return v


def _host(h, name):
    """HostOptions (configuration.rs:690-716)."""
    where = f"hosts.{name}"
    _check_keys(h, ["network_node_id", "processes", "ip_addr", "bandwidth_down", "bandwidth_up",
                    "host_options"], [where])
    for req in ("network_node_id", "processes"):
        if req not in h:
            raise ConfigError(f"{where}: missing field `{req}`")
    procs = h["processes"]
    if not isinstance(procs, list):
        raise ConfigError(f"{where}.processes: invalid type: expected a sequence")
    ho = h.get("host_options")
    return {
        "network_node_id": _p_u32(h["network_node_id"], f"{where}.network_node_id"),
        "processes": [_process(p, f"{where}.processes[{i}]") for i, p in enumerate(procs)],
        "ip_addr": None if h.get("ip_addr") is None else _ipv4(h["ip_addr"], f"{where}.ip_addr"),
        "bandwidth_down": None if h.get("bandwidth_down") is None else Unit.from_yaml("bits", h["bandwidth_down"], f"{where}.bandwidth_down"),
        "bandwidth_up": None if h.get("bandwidth_up") is None else Unit.from_yaml("bits", h["bandwidth_up"], f"{where}.bandwidth_up"),
        "host_options": _section({} if ho is None else ho, HOST_DEFAULTS, [where, "host_options"], False),
    }


@dataclass
class ConfigFile:
    """ConfigFileOptions (configuration.rs:92-109) after deserialization."""
    general: dict
    network: dict
    host_option_defaults: dict
    experimental: dict
    hosts: dict  # hostname -> host dict, sorted by hostname (BTreeMap)


def parse_config_file(doc) -> ConfigFile:
    _check_keys(doc, ["general", "network", "host_option_defaults", "experimental", "hosts"], [])
    for req in ("general", "network", "hosts"):
        if req not in doc:
            raise ConfigError(f"missing field `{req}`")
    general = _section(doc["general"], GENERAL, ["general"], True)
    network = _section(doc["network"], NETWORK, ["network"], True)
    if doc["network"].get("graph") is not None:
        network["graph"] = _graph(doc["network"]["graph"], "network.graph")
    hod = doc.get("host_option_defaults")
    host_option_defaults = _section({} if hod is None else hod, HOST_DEFAULTS, ["host_option_defaults"], False)
    exp = doc.get("experimental")
    experimental = _section({} if exp is None else exp, EXPERIMENTAL, ["experimental"], True)
    hosts_in = doc["hosts"]
    if not isinstance(hosts_in, dict):
        raise ConfigError("hosts: invalid type: expected a map")
    hosts = {}
    for k in hosts_in:
        _hostname(k)
    for k in sorted(hosts_in):
        hosts[k] = _host(hosts_in[k], k)
    return ConfigFile(general, network, host_option_defaults, experimental, hosts)


# --------------------------------------------------------------------------------------
# Command line (clap over CliOptions, configuration.rs:33-89) and the merge
# --------------------------------------------------------------------------------------

_SECTIONS = {"general": GENERAL, "network": NETWORK, "host_option_defaults": HOST_DEFAULTS,
             "experimental": EXPERIMENTAL}


def _cli_table():
    t = {}
    for sec, schema in _SECTIONS.items():
        for name, parse, _, nullable in schema:
            if parse is None:
                continue
            flag = _CLI_RENAME.get((sec, name), name.replace("_", "-"))
            t[flag] = (sec, name, parse, nullable)
    return t


def _cli_value(name, parse, nullable, text):
    """clap value_parser = FromStr of the field type; NullableOption accepts "null"."""
    if nullable and text == "null":
        return NULL
    return parse.cli(text, f"--{name.replace('_', '-')}")


@dataclass
class CliOptions:
    config: str | None = None
    debug_hosts: set = field(default_factory=set)
    show_config: bool = False
    sections: dict = field(default_factory=lambda: {s: {} for s in _SECTIONS})


def parse_cli(argv) -> CliOptions:
    """The override subset of `shadow [OPTIONS] <CONFIG>`: --long value, --long=value,
    -x value, -xVALUE. Flags not on the packet path's schema raise like clap does."""
    table = _cli_table()
    out = CliOptions()
    i = 0
    argv = list(argv)
    while i < len(argv):
        a = argv[i]
        if a.startswith("--") and len(a) > 2:
            key, eq, val = a[2:].partition("=")
            if key in ("show-config", "gdb", "shm-cleanup", "show-build-info"):
                if key == "show-config":
                    out.show_config = True
                i += 1
                continue
            if key == "debug-hosts":
                if not eq:
                    i += 1
                    val = argv[i] if i < len(argv) else None
                if val is None:
                    raise ConfigError("--debug-hosts: a value is required")
                out.debug_hosts = {x for x in val.split(",") if x}
                i += 1
                continue
            if key not in table:
                raise ConfigError(f"unexpected argument '--{key}' found")
            sec, name, parse, nullable = table[key]
        elif a.startswith("-") and len(a) >= 2 and a != "-":
            if a[1] not in _CLI_SHORT:
                raise ConfigError(f"unexpected argument '{a}' found")
            sec, name = _CLI_SHORT[a[1]]
            parse, nullable = next((p, nl) for n, p, _, nl in _SECTIONS[sec] if n == name)
            val = a[2:].lstrip("=")
            eq = bool(val)
        else:
            if out.config is not None:
                raise ConfigError(f"unexpected argument '{a}' found")
            out.config = a
            i += 1
            continue
        if not eq:
            i += 1
            if i >= len(argv):
                raise ConfigError(f"a value is required for '--{name.replace('_', '-')}'")
            val = argv[i]
        out.sections[sec][name] = _cli_value(name, parse, nullable, val)
        i += 1
    return out


def _with_defaults(base: dict, default: dict) -> dict:
    """merge::option::overwrite_none: unset (None) fields of `base` take `default`'s."""
    return {k: (default.get(k) if base.get(k) is None else base[k]) for k in default}


def _denull(v):
    return None if v is NULL else v


@dataclass
class ConfigOptions:
    """ConfigOptions (configuration.rs:111-154): the file merged with the command line."""
    general: dict
    network: dict
    experimental: dict
    hosts: dict

    @classmethod
    def new(cls, cf: ConfigFile, cli: CliOptions | None = None) -> "ConfigOptions":
        cli = cli or CliOptions()
        hod = _with_defaults(cf.host_option_defaults, {n: d for n, _, d, _ in HOST_DEFAULTS})
        full = lambda sec: {n: cli.sections[sec].get(n) for n, *_ in _SECTIONS[sec]}  # noqa: E731
        general = _with_defaults(full("general"), cf.general)
        network = _with_defaults(full("network"), cf.network)
        hod = _with_defaults(full("host_option_defaults"), hod)
        experimental = _with_defaults(full("experimental"), cf.experimental)
        hosts = {}
        for name, h in cf.hosts.items():
            h = dict(h)
            h["host_options"] = _with_defaults(h["host_options"], hod)
            hosts[name] = h
        return cls(general, network, experimental, hosts)

    def processed(self) -> dict:
        """The serialized form the reference writes as processed-config.yaml
        (core/manager.rs:253): units in Display form, NullableOption::Null and None as null."""
        def ser(v):
            if isinstance(v, Unit):
                return str(v)
            if v is NULL:
                return None
            if isinstance(v, dict):
                return {k: ser(x) for k, x in v.items()}
            if isinstance(v, list):
                return [ser(x) for x in v]
            return v
        hosts = {}
        for name, h in self.hosts.items():
            hosts[name] = {
                "network_node_id": h["network_node_id"],
                "processes": [ser(p) for p in h["processes"]],
                "ip_addr": h["ip_addr"],
                "bandwidth_down": ser(h["bandwidth_down"]),
                "bandwidth_up": ser(h["bandwidth_up"]),
                "host_options": ser(h["host_options"]),
            }
        return {"general": ser(self.general), "network": ser(self.network),
                "experimental": ser(self.experimental), "hosts": hosts}


def load(path=None, *, text=None, argv=()) -> ConfigOptions:
    """shadow.rs:96-100: the config file (path, or text) merged with command-line flags."""
    cli = parse_cli(argv)
    if text is None:
        path = path or cli.config
        if path is None:
            raise ConfigError("no configuration file given")
        try:
            with open("/dev/stdin" if path == "-" else path, encoding="utf-8") as f:
                text = f.read()
        except OSError as e:
            raise ConfigError(f"Could not open config file: {e}") from None
    return ConfigOptions.new(parse_config_file(load_yaml(text)), cli)


# --------------------------------------------------------------------------------------
# SimConfig::new (sim_config.rs:47-164) -> libsgn inputs
# --------------------------------------------------------------------------------------

# configuration.rs:1367-1381 (the text is data: the built-in graph of `type: 1_gbit_switch`)
ONE_GBIT_SWITCH_GRAPH = """graph [
  directed 0
  node [
    id 0
    host_bandwidth_up "1 Gbit"
    host_bandwidth_down "1 Gbit"
  ]
  edge [
    source 0
    target 0
    latency "1 ms"
    packet_loss 0.0
  ]
]"""


def _tilde(p):
    """tilde_expansion (utility/mod.rs): a leading "~/" is the home directory."""
    return os.path.expanduser(p) if p.startswith("~/") or p == "~" else p


def load_network_graph(graph: dict, base_dir=None) -> str:
    """network/graph/mod.rs:478-507."""
    if graph["type"] == "1_gbit_switch":
        return ONE_GBIT_SWITCH_GRAPH
    if "inline" in graph:
        return graph["inline"]
    path = _tilde(graph["file"]["path"])
    if base_dir and not os.path.isabs(path):
        path = os.path.join(base_dir, path)
    try:
        if graph["file"]["compression"] == "xz":
            with open(path, "rb") as f:
                data = lzma.decompress(f.read(), format=lzma.FORMAT_XZ)
            return data.decode("utf-8")
        with open(path, encoding="utf-8") as f:
            return f.read()
    except (OSError, lzma.LZMAError, UnicodeDecodeError) as e:
        raise ConfigError(f"Failed to load the network graph: {e}") from None


@dataclass
class SimSetup:
    """Everything libsgn needs to start the packet core, in HostId (= hostname) order."""
    names: list
    graph: sgn.GraphArrays
    used_nodes: np.ndarray
    hosts: sgn.HostArrays
    use_shortest_path: bool
    stop_time_ns: int
    bootstrap_end_ns: int
    runahead_ns: int  # 0 = None (no lower bound, runahead.rs:55)
    use_dynamic_runahead: bool
    qdisc: int
    seed: int
    process_start_ns: list  # per host: start times of its processes (informational)

    def sim_config(self, **engine):
        """sgn_sim_config with the engine capacities (out_fifo_cap, codel_cap, event_capacity ...)
        supplied by the caller."""
        return sgn.make_config(self.stop_time_ns, bootstrap_end_ns=self.bootstrap_end_ns,
                               runahead_ns=self.runahead_ns, dynamic=self.use_dynamic_runahead,
                               qdisc=self.qdisc, **engine)


def sim_setup(cfg: ConfigOptions, base_dir=None, debug_hosts=(), lib=None) -> SimSetup:
    g = cfg.general
    if g["stop_time"] is None:
        raise ConfigError("general.stop_time is required")
    stop_ns = g["stop_time"].base()
    names = list(cfg.hosts)  # BTreeMap order
    starts = []
    for name, h in cfg.hosts.items():  # build_host / build_process checks (sim_config.rs:294-326)
        st = []
        for p in h["processes"]:
            s = p["start_time"].base()
            if s >= stop_ns:
                raise ConfigError(f"Failed to configure host '{name}': Process start time "
                                  f"'{p['start_time']}' must be earlier than the simulation stop "
                                  f"time '{g['stop_time']}'")
            if p["shutdown_time"] is not None:
                sh = p["shutdown_time"].base()
                if s >= sh:
                    raise ConfigError(f"Failed to configure host '{name}': Process start time "
                                      f"'{p['start_time']}' must be earlier than its shutdown_time "
                                      f"time '{p['shutdown_time']}'")
                if sh >= stop_ns:
                    raise ConfigError(f"Failed to configure host '{name}': Process shutdown_time "
                                      f"'{p['shutdown_time']}' must be earlier than the simulation "
                                      f"stop time '{g['stop_time']}'")
            st.append(s)
        starts.append(st)
    if not names:
        raise ConfigError("The configuration did not contain any hosts")
    if cfg.network["graph"] is None:
        raise ConfigError("network.graph is required")
    text = load_network_graph(cfg.network["graph"], base_dir)
    try:
        graph, node_bw = sgn.gml_parse(text, lib)
    except sgn.SgnError as e:
        raise ConfigError(f"Failed to parse the network graph: {e}") from None
    index = {int(n): i for i, n in enumerate(graph.node_id)}
    n = len(names)
    node = np.zeros(n, np.uint32)
    up = np.zeros(n, np.uint64)
    down = np.zeros(n, np.uint64)
    explicit = {}
    for i, (name, h) in enumerate(cfg.hosts.items()):
        nid = h["network_node_id"]
        if nid not in index:
            raise ConfigError(f"The network node id {nid} for host '{name}' does not exist")
        node[i] = nid
        g_up, g_down = node_bw[index[nid]]
        # sim_config.rs:249-254: both host-side values come from bandwidth_down
        h_bw = None if h["bandwidth_down"] is None else h["bandwidth_down"].base()
        d = h_bw if h_bw is not None else g_down
        u = h_bw if h_bw is not None else g_up
        if d is None:
            raise ConfigError(f"No downstream bandwidth provided for host '{name}'")
        if u is None:
            raise ConfigError(f"No upstream bandwidth provided for host '{name}'")
        down[i], up[i] = d, u
        if h["ip_addr"] is not None:
            explicit[i] = int(ipaddress.IPv4Address(h["ip_addr"]))
    for hn in debug_hosts:
        if hn not in cfg.hosts:
            raise ConfigError(f"The host to debug '{hn}' doesn't exist")
    try:
        ips = sgn.assign_ips(n, explicit, lib)
    except sgn.SgnError as e:
        raise ConfigError(f"Failed to assign IP addresses: {e}") from None
    seeds = sgn.derive_seeds(g["seed"], names, lib)
    runahead = _denull(cfg.experimental["runahead"])
    boot = g["bootstrap_end_time"]
    return SimSetup(
        names=names, graph=graph, used_nodes=np.unique(node),
        hosts=sgn.HostArrays(ips, node, up, down, seeds),
        use_shortest_path=bool(cfg.network["use_shortest_path"]),
        stop_time_ns=stop_ns, bootstrap_end_ns=0 if boot is None else boot.base(),
        runahead_ns=0 if runahead is None else runahead.base(),
        use_dynamic_runahead=bool(cfg.experimental["use_dynamic_runahead"]),
        qdisc=sgn.QDISC_ROUND_ROBIN if cfg.experimental["interface_qdisc"] == "round-robin" else sgn.QDISC_FIFO,
        seed=g["seed"], process_start_ns=starts)
