"""Exact reconstruction of the reference's error values from (err_code, args).

Each GPD_E_* code names one `return ...error` site of the reference decoders
(include/gpd.h lists the file:line of each); the text below is the format
string at that site, so `str(err)` equals the Go `err.Error()`.
"""
from __future__ import annotations

from .layers import ip_protocol_name, layer_type_name

# code -> (format, number of args, arg formatter)
_FORMATS = {
    1: "Ethernet packet too small",
    2: "802.1Q tag length {0} too short",
    3: "Invalid ip4 header. Length {0} less than 20",
    4: "Invalid (too small) IP length ({0} < 20)",
    5: "Invalid (too small) IP header length ({0} < 5)",
    6: "Invalid IP header length > IP length ({0} > {1})",
    7: "Not all IP header bytes available",
    8: "Invalid ip4 option length. Length {0} less than 2",
    9: "IP option length exceeds remaining IP header size, option type {0} length {1}",
    10: "Invalid IP option type {0} length {1}. Must be greater than 2",
    11: "Invalid ip6 header. Length {0} less than 40",
    12: "Invalid ip6-extension header. Length {0} less than 2",
    13: "Invalid ip6-extension header. Length {0} less than specified length {1}",
    14: "IPv6 header option too small",
    15: "IPv6 header TLV option too small",
    16: "Jumbo length TLV data must have length 4",
    17: "Jumbo length cannot be less than 65536",
    18: "IPv6 has jumbo length and IPv6 length is not 0",
    19: "IPv6 length 0, but HopByHop header does not have jumbogram option",
    20: "IPv6 length 0, but next header is {0p}, not HopByHop",
    21: "Invalid TCP header. Length {0} less than 20",
    22: "Invalid TCP data offset {0} < 5",
    23: "TCP data offset greater than packet length",
    24: "Invalid TCP option length. Length {0} less than 2",
    25: "Invalid TCP option length {0} < 2",
    26: "Invalid TCP option length {0} exceeds remaining {1} bytes",
    27: "Invalid UDP header. Length {0} less than 8",
    28: "UDP packet too small: {0} bytes",
    29: "vxlan packet too small",
    30: "ICMP layer less then 8 bytes for ICMPv4 packet",
    31: "LLC header too small",
}

ERR_CODE_NAMES = {
    1: "ETH_TOO_SMALL", 2: "DOT1Q_TOO_SHORT", 3: "IP4_TOO_SHORT", 4: "IP4_LENGTH_LT20",
    5: "IP4_IHL_LT5", 6: "IP4_IHL_GT_LENGTH", 7: "IP4_HDR_TRUNC", 8: "IP4_OPT_LT2",
    9: "IP4_OPT_EXCEEDS", 10: "IP4_OPT_LE2", 11: "IP6_TOO_SHORT", 12: "IP6EXT_LT2",
    13: "IP6EXT_LT_SPEC", 14: "IP6_TLV_LT2", 15: "IP6_TLV_TRUNC", 16: "IP6_JUMBO_TLV_LEN",
    17: "IP6_JUMBO_TOO_SMALL", 18: "IP6_JUMBO_AND_LEN", 19: "IP6_LEN0_NO_JUMBO",
    20: "IP6_LEN0_NOT_HBH", 21: "TCP_TOO_SHORT", 22: "TCP_DOFF_LT5", 23: "TCP_DOFF_GT_LEN",
    24: "TCP_OPT_LT2_REM", 25: "TCP_OPT_LEN_LT2", 26: "TCP_OPT_EXCEEDS", 27: "UDP_TOO_SHORT",
    28: "UDP_LEN_TOO_SMALL", 29: "VXLAN_TOO_SMALL", 30: "ICMP4_TOO_SMALL", 31: "LLC_TOO_SMALL",
}


class DecodeError(Exception):
    """A layer's DecodeFromBytes error (the reference returns errors.New / fmt.Errorf)."""

    def __init__(self, code: int, arg0: int = 0, arg1: int = 0):
        self.code, self.arg0, self.arg1 = int(code), int(arg0), int(arg1)
        super().__init__(decode_error_text(self.code, self.arg0, self.arg1))

    def Error(self) -> str:
        return str(self)


class UnsupportedLayerType(Exception):
    """parser.go:318-326."""

    def __init__(self, layer_type: int):
        self.layer_type = int(layer_type)
        super().__init__(f"No decoder for layer type {layer_type_name(self.layer_type)}")

    def Error(self) -> str:
        return str(self)


def decode_error_text(code: int, a0: int = 0, a1: int = 0) -> str:
    fmt = _FORMATS.get(int(code))
    if fmt is None:
        return f"gpd: unknown error code {code}"
    return fmt.replace("{0p}", ip_protocol_name(a0)).format(a0, a1)
