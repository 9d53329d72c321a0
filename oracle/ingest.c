/* TEST INFRASTRUCTURE ONLY (see svo_oracle.h): colour ingest restated.
 *
 * R:include/async_image_loader.h:63-69 reads KITTI's colour images with
 * cv::imread (8UC3, BGR order) and converts them with
 * cv::cvtColor(COLOR_BGR2GRAY). OpenCV imgproc color_rgb RGB2Gray<uchar>:
 * three 256-entry tables b*B2Y, g*G2Y, (1 << 13) + r*R2Y with R2Y = 4899,
 * G2Y = 9617, B2Y = 1868 and yuv_shift = 14; gray = sum >> 14. */
#include "svo_oracle.h"

void svo_oracle_bgr2gray(const uint8_t* bgr, int w, int h, int stride, uint8_t* gray) {
    for (int y = 0; y < h; y++) {
        const uint8_t* s = bgr + (long)y * stride;
        for (int x = 0; x < w; x++) {
            const int b = s[3 * x], g = s[3 * x + 1], r = s[3 * x + 2];
            gray[(long)y * w + x] = (uint8_t)((b * 1868 + g * 9617 + (1 << 13) + r * 4899) >> 14);
        }
    }
}
