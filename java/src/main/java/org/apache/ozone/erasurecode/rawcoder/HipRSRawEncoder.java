package org.apache.ozone.erasurecode.rawcoder;

import org.apache.hadoop.hdds.client.ECReplicationConfig;

/** RS raw encoder on the GPU (libozec): bit-exact with RSRawEncoder (EC/rawcoder/RSRawEncoder.java). */
public class HipRSRawEncoder extends AbstractHipRawEncoder {
  public HipRSRawEncoder(ECReplicationConfig config) {
    super(config, OzecNative.CODEC_RS);
  }
}
