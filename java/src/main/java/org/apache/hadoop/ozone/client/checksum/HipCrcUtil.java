package org.apache.hadoop.ozone.client.checksum;

import java.io.IOException;

import org.apache.hadoop.util.DataChecksum;
import org.apache.ozone.erasurecode.rawcoder.OzecNative;

/**
 * CrcUtil.getMonomial / CrcUtil.compose (OC/CrcUtil.java:74-127) over ozec_crc_monomial / ozec_crc_compose, for the
 * two polynomials Ozone uses (CrcUtil.GZIP_POLYNOMIAL, CrcUtil.CASTAGNOLI_POLYNOMIAL: CrcUtil.java:35-36), with the
 * reference's IllegalArgumentException for a negative length.  Byte helpers (intToBytes, readInt, ...) stay
 * CrcUtil's.  OC/ = hadoop-ozone/common/src/main/java/org/apache/hadoop/ozone/client/checksum/
 */
public final class HipCrcUtil {
  private HipCrcUtil() {
  }

  /** x^(8 * lengthBytes) mod the polynomial, in CrcUtil's reversed representation. */
  public static int getMonomial(long lengthBytes, int mod) {
    return OzecNative.crcMonomial(typeOfPolynomial(mod), lengthBytes);
  }

  /** crcA * x^(8 * lengthB) xor crcB: the CRC of A || B. */
  public static int compose(int crcA, int crcB, long lengthB, int mod) {
    return OzecNative.crcCompose(typeOfPolynomial(mod), crcA, crcB, lengthB);
  }

  /** CrcUtil.getCrcPolynomialForType's types (:53-64) as libozec checksum types. */
  static int checksumType(DataChecksum.Type type) throws IOException {
    switch (type) {
      case CRC32:
        return OzecNative.CHECKSUM_CRC32;
      case CRC32C:
        return OzecNative.CHECKSUM_CRC32C;
      default:
        throw new IOException("No CRC polynomial could be associated with type: " + type);
    }
  }

  private static int typeOfPolynomial(int mod) {
    if (mod == CrcUtil.GZIP_POLYNOMIAL) {
      return OzecNative.CHECKSUM_CRC32;
    }
    if (mod == CrcUtil.CASTAGNOLI_POLYNOMIAL) {
      return OzecNative.CHECKSUM_CRC32C;
    }
    throw new IllegalArgumentException("libozec composes CRC32 and CRC32C only, not polynomial 0x"
        + Integer.toHexString(mod));
  }
}
