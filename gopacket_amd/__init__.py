"""gopacket_amd: gopacket's DecodingLayerParser fast path on MI355X."""
