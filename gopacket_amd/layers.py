"""LayerType numbers, enum names and the reference's default dispatch tables.

Restates (as data) what gopacket's init code builds:
  * LayerType IDs .......... decode.go:105-116, layers/layertypes.go:14-154
  * EthernetType -> LayerType  layers/enums.go:304-321 (unknown -> LayerTypeZero,
                               layers/enums_generated.go:93-101)
  * IPProtocol -> LayerType .. layers/enums.go:323-345
  * TCP/UDP port -> LayerType  layers/ports.go:62-74, 105-122 (0 means Payload,
                               ports.go:54-60, 97-103)
Tables are mutable like the reference's globals (RegisterTCPPortLayerType,
ports.go:78-80; RegisterUDPPortLayerType, ports.go:126-128); a parser snapshots
them when it is created (see parser.DecodingLayerParser.reload_tables).
"""
from __future__ import annotations

import numpy as np

from ._names import IPPROTOCOL_NAMES, LAYERTYPE_NAMES

# --- LayerType numbers -------------------------------------------------------
LayerTypeZero = 0
LayerTypeDecodeFailure = 1
LayerTypePayload = 2
LayerTypeFragment = 3
LayerTypeARP = 10
LayerTypeCiscoDiscovery = 11
LayerTypeEthernetCTP = 12
LayerTypeDot1Q = 15
LayerTypeEtherIP = 16
LayerTypeEthernet = 17
LayerTypeGRE = 18
LayerTypeICMPv4 = 19
LayerTypeIPv4 = 20
LayerTypeIPv6 = 21
LayerTypeLLC = 22
LayerTypeSNAP = 23
LayerTypeMPLS = 24
LayerTypePPP = 25
LayerTypePPPoE = 26
LayerTypeRUDP = 27
LayerTypeSCTP = 28
LayerTypeTCP = 44
LayerTypeUDP = 45
LayerTypeIPv6HopByHop = 46
LayerTypeIPv6Routing = 47
LayerTypeIPv6Fragment = 48
LayerTypeIPv6Destination = 49
LayerTypeIPSecAH = 50
LayerTypeIPSecESP = 51
LayerTypeUDPLite = 52
LayerTypeEAPOL = 56
LayerTypeICMPv6 = 57
LayerTypeLinkLayerDiscovery = 58
LayerTypeNortelDiscovery = 61
LayerTypeIGMP = 62
LayerTypeDNS = 107
LayerTypeSFlow = 114
LayerTypeVXLAN = 116
LayerTypeNTP = 117
LayerTypeDHCPv4 = 118
LayerTypeVRRP = 119
LayerTypeGeneve = 120
LayerTypeSTP = 121
LayerTypeBFD = 122
LayerTypeOSPF = 123
LayerTypeGTPv1U = 129
LayerTypeSIP = 133
LayerTypeDHCPv6 = 134
LayerTypeTLS = 140
LayerTypeModbusTCP = 141
LayerTypeRMCP = 142
LayerTypeERSPANII = 145
LayerTypeRADIUS = 146
LayerTypeAGUEVar0 = 147
LayerTypeAPSP = 149

# LayerClassIPv6Extension, layers/layertypes.go:193-198
LayerClassIPv6Extension = (LayerTypeIPv6HopByHop, LayerTypeIPv6Routing,
                           LayerTypeIPv6Fragment, LayerTypeIPv6Destination)

# EndpointType numbers, layers/endpoints.go:20-35
EndpointIPv4 = 1
EndpointIPv6 = 2
EndpointMAC = 3
EndpointTCPPort = 4
EndpointUDPPort = 5

# 4-bit layer codes used in the packed `layers` output (include/gpd.h GPD_C_*)
CODE_TO_LAYERTYPE = (0, LayerTypeEthernet, LayerTypeDot1Q, LayerTypeIPv4, LayerTypeIPv6,
                     LayerTypeIPv6HopByHop, LayerTypeIPv6Routing, LayerTypeIPv6Fragment,
                     LayerTypeIPv6Destination, LayerTypeTCP, LayerTypeUDP, LayerTypeVXLAN,
                     LayerTypePayload, LayerTypeFragment, LayerTypeICMPv4, LayerTypeLLC)
LAYERTYPE_TO_CODE = {lt: c for c, lt in enumerate(CODE_TO_LAYERTYPE) if lt}


def layer_type_name(t: int) -> str:
    """LayerType.String(), layertype.go:101-112 (unregistered -> decimal)."""
    s = LAYERTYPE_NAMES.get(int(t), "")
    return s if s else str(int(t))


def ip_protocol_name(p: int) -> str:
    """IPProtocol.String(), enums_generated.go:146-148 (unknown -> 'UnknownIPProtocol')."""
    return IPPROTOCOL_NAMES.get(int(p), "UnknownIPProtocol")


# --- default dispatch tables ---------------------------------------------------
_ETHERTYPE_DEFAULTS = {  # layers/enums.go:304-321
    0x0000: LayerTypeLLC, 0x0800: LayerTypeIPv4, 0x86DD: LayerTypeIPv6, 0x0806: LayerTypeARP,
    0x8100: LayerTypeDot1Q, 0x880B: LayerTypePPP, 0x8863: LayerTypePPPoE, 0x8864: LayerTypePPPoE,
    0x9000: LayerTypeEthernetCTP, 0x2000: LayerTypeCiscoDiscovery,
    0x01A2: LayerTypeNortelDiscovery, 0x88CC: LayerTypeLinkLayerDiscovery,
    0x8847: LayerTypeMPLS, 0x8848: LayerTypeMPLS, 0x888E: LayerTypeEAPOL,
    0x88A8: LayerTypeDot1Q, 0x6558: LayerTypeEthernet, 0x88BE: LayerTypeERSPANII,
}
_IPPROTO_DEFAULTS = {  # layers/enums.go:323-345
    4: LayerTypeIPv4, 6: LayerTypeTCP, 17: LayerTypeUDP, 1: LayerTypeICMPv4, 58: LayerTypeICMPv6,
    132: LayerTypeSCTP, 41: LayerTypeIPv6, 94: LayerTypeIPv4, 97: LayerTypeEtherIP,
    27: LayerTypeRUDP, 47: LayerTypeGRE, 0: LayerTypeIPv6HopByHop, 43: LayerTypeIPv6Routing,
    44: LayerTypeIPv6Fragment, 60: LayerTypeIPv6Destination, 89: LayerTypeOSPF,
    51: LayerTypeIPSecAH, 50: LayerTypeIPSecESP, 136: LayerTypeUDPLite, 137: LayerTypeMPLS,
    59: LayerTypePayload, 2: LayerTypeIGMP, 112: LayerTypeVRRP,
}
_TCP_PORT_DEFAULTS = {  # layers/ports.go:62-74
    53: LayerTypeDNS, 443: LayerTypeTLS, 502: LayerTypeModbusTCP, 636: LayerTypeTLS,
    989: LayerTypeTLS, 990: LayerTypeTLS, 992: LayerTypeTLS, 993: LayerTypeTLS,
    994: LayerTypeTLS, 995: LayerTypeTLS, 5061: LayerTypeTLS,
}
_UDP_PORT_DEFAULTS = {  # layers/ports.go:105-122
    53: LayerTypeDNS, 123: LayerTypeNTP, 4789: LayerTypeVXLAN, 67: LayerTypeDHCPv4,
    68: LayerTypeDHCPv4, 546: LayerTypeDHCPv6, 547: LayerTypeDHCPv6, 666: LayerTypeAGUEVar0,
    1000: LayerTypeAPSP, 5060: LayerTypeSIP, 6343: LayerTypeSFlow, 6081: LayerTypeGeneve,
    3784: LayerTypeBFD, 2152: LayerTypeGTPv1U, 623: LayerTypeRMCP, 1812: LayerTypeRADIUS,
}


def _table(size, entries):
    t = np.zeros(size, dtype=np.uint16)
    for k, v in entries.items():
        t[k] = v
    return t


class DispatchTables:
    """The four enum->LayerType tables a DecodingLayerParser consults."""

    def __init__(self):
        self.ethertype = _table(65536, _ETHERTYPE_DEFAULTS)
        self.ipproto = _table(256, _IPPROTO_DEFAULTS)
        self.tcp_port = _table(65536, _TCP_PORT_DEFAULTS)
        self.udp_port = _table(65536, _UDP_PORT_DEFAULTS)

    def copy(self) -> "DispatchTables":
        c = DispatchTables.__new__(DispatchTables)
        c.ethertype = self.ethertype.copy()
        c.ipproto = self.ipproto.copy()
        c.tcp_port = self.tcp_port.copy()
        c.udp_port = self.udp_port.copy()
        return c


# The process-wide tables, like the reference's package globals.
TABLES = DispatchTables()


def RegisterTCPPortLayerType(port: int, layer_type: int) -> None:
    """layers/ports.go:78-80."""
    TABLES.tcp_port[int(port) & 0xFFFF] = int(layer_type)


def RegisterUDPPortLayerType(port: int, layer_type: int) -> None:
    """layers/ports.go:126-128."""
    TABLES.udp_port[int(port) & 0xFFFF] = int(layer_type)


def SetEthernetTypeLayerType(ethertype: int, layer_type: int) -> None:
    """EthernetTypeMetadata[t].LayerType = lt (layers/enums.go:288-321 documents the override)."""
    TABLES.ethertype[int(ethertype) & 0xFFFF] = int(layer_type)


def SetIPProtocolLayerType(proto: int, layer_type: int) -> None:
    """IPProtocolMetadata[p].LayerType = lt (layers/enums.go:323-345)."""
    TABLES.ipproto[int(proto) & 0xFF] = int(layer_type)
