package org.apache.ozone.erasurecode.rawcoder;

import org.apache.hadoop.hdds.client.ECReplicationConfig;

/**
 * Factory of the GPU RS coders (RawErasureCoderFactory, EC/rawcoder/RawErasureCoderFactory.java:29-56), registered
 * through META-INF/services of its own jar.  The coder constructors throw without a GPU or libozec_jni, so
 * CodecUtil.createRawEncoderWithFallback moves on to the next coder (CodecUtil.java:62-78).
 */
public class HipRSRawErasureCoderFactory implements RawErasureCoderFactory {
  public static final String CODER_NAME = "rs_hip";

  @Override
  public RawErasureEncoder createEncoder(ECReplicationConfig config) {
    return new HipRSRawEncoder(config);
  }

  @Override
  public RawErasureDecoder createDecoder(ECReplicationConfig config) {
    return new HipRSRawDecoder(config);
  }

  @Override
  public String getCoderName() {
    return CODER_NAME;
  }

  @Override
  public String getCodecName() {
    return ECReplicationConfig.EcCodec.RS.name().toLowerCase();
  }
}
