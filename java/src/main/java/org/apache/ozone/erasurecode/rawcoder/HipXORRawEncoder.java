package org.apache.ozone.erasurecode.rawcoder;

import org.apache.hadoop.hdds.client.ECReplicationConfig;

/** XOR raw encoder on the GPU (libozec): bit-exact with XORRawEncoder (EC/rawcoder/XORRawEncoder.java). */
public class HipXORRawEncoder extends AbstractHipRawEncoder {
  public HipXORRawEncoder(ECReplicationConfig config) {
    super(config, OzecNative.CODEC_XOR);
  }
}
