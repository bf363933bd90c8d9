package org.apache.ozone.erasurecode.rawcoder;

import org.apache.hadoop.hdds.client.ECReplicationConfig;

/** RS raw decoder on the GPU (libozec): bit-exact with RSRawDecoder (EC/rawcoder/RSRawDecoder.java). */
public class HipRSRawDecoder extends AbstractHipRawDecoder {
  public HipRSRawDecoder(ECReplicationConfig config) {
    super(config, OzecNative.CODEC_RS);
  }
}
