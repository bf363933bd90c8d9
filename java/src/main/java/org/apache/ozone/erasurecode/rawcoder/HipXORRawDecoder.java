package org.apache.ozone.erasurecode.rawcoder;

import org.apache.hadoop.hdds.client.ECReplicationConfig;

/** XOR raw decoder on the GPU (libozec): bit-exact with XORRawDecoder (EC/rawcoder/XORRawDecoder.java). */
public class HipXORRawDecoder extends AbstractHipRawDecoder {
  public HipXORRawDecoder(ECReplicationConfig config) {
    super(config, OzecNative.CODEC_XOR);
  }
}
