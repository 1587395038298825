/*
 * rtc_scene.h — host-side scene input for the render path (C-ABI).
 *
 * Mirrors the reference's scene construction API so a caller can go from the
 * YAML scene files to the descriptor tables rt_scene_upload() takes:
 *   load_scene_description(path) -> (World, Camera)
 *       ray-tracer-cli/src/scene_loader.rs:361-367   -> rt_scene_load_yaml
 *   Camera::new + set_transformation(view_transform(from, to, up))
 *       scene_loader.rs:255-266, camera.rs:25-49/124-127,
 *       transformations.rs:75-87                      -> rt_camera_make
 *   Matrix<4>::inverse  primitives/matrix.rs:247-258  -> rt_matrix_inverse
 *   Canvas::to_png_file / to_ppm_file  canvas.rs:75-137 -> rt_image_write
 *   Color::clamped + u8 cast  canvas.rs:81, 117-123   -> rt_canvas_quantize
 * All arithmetic is f64 and follows the reference's operation order, so the
 * tables are bit-identical to what the reference holds after loading.
 * Pure host code: none of these functions needs a GPU.
 */
#ifndef RTC_SCENE_H
#define RTC_SCENE_H

#include "rtc.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_scene rt_scene;

typedef struct rt_scene_view {
    const rt_shape_desc* shapes;
    uint32_t n_shapes;
    const rt_material_desc* materials;
    uint32_t n_materials;
    const rt_pattern_desc* patterns;
    uint32_t n_patterns;
    const rt_light_desc* lights;
    uint32_t n_lights;
    rt_camera_desc camera;
    /* Shapes equal by value to an earlier shape (shape.rs:34-38).  The
     * reference's containers walk identifies shapes by value
     * (intersection.rs:47); rt_scene_upload gives value-equal shapes one
     * identity class so the device walk does the same. */
    uint32_t duplicate_shapes;
} rt_scene_view;

/* load_scene_description (scene_loader.rs:361-367).  RT_ERR_IO on a parse
 * error, with the reason in rt_last_error(). */
int rt_scene_load_yaml(const char* path, rt_scene** out);
int rt_scene_load_yaml_text(const char* text, rt_scene** out);
int rt_scene_view_get(const rt_scene* scene, rt_scene_view* view);
void rt_scene_free(rt_scene* scene);

/* Camera::new(width, height, fov) + set_transformation(view_transform(...)) */
int rt_camera_make(uint32_t width, uint32_t height, double field_of_view,
                   const double from[3], const double to[3], const double up[3],
                   rt_camera_desc* out);

/* Re-run Camera::new for a new canvas size, keeping fov and transform —
 * equivalent to editing the YAML camera width/height. */
int rt_camera_resize(rt_camera_desc* camera, uint32_t width, uint32_t height);

/* Camera::set_transformation (camera.rs:124-127): store the inverse of the
 * row-major `transform` and update the origin (camera.rs:114-116). */
int rt_camera_set_transform(rt_camera_desc* camera, const double transform[16]);

/* Matrix<4>::inverse, row-major 16 doubles. */
int rt_matrix_inverse(const double m[16], double out[16]);

/* Canvas::to_png_file / to_ppm_file (canvas.rs:75-137) for an 8-bit frame
 * (rt_render with RT_OUT_U8, row-major RGB, y = 0 at the top): a path ending
 * in ".png" (any case) gets an RGB8 PNG (filter None, best deflate, as the
 * reference writes), anything else the reference's P3 text byte for byte
 * (canvas.rs:75-97: 5 pixels per line across row boundaries, channels
 * right-aligned to width 3, no trailing newline).  The parent directories
 * are created first (canvas.rs:99-105).  RT_ERR_IO on a write failure.
 * Host only. */
int rt_image_write(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height);

enum {
    RT_IMAGE_AUTO = 0,        /* by extension, as rt_image_write */
    RT_IMAGE_PNG = 1,         /* Canvas::to_png_file */
    RT_IMAGE_PPM = 2,         /* Canvas::to_ppm_file: P3 text, the reference's bytes */
    RT_IMAGE_PPM_BINARY = 3   /* P6 (not in the reference): the same pixels in 1/4 of the bytes */
};
int rt_image_write_format(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height, int format);

/* The canvas's 8-bit quantization on the host (canvas.rs:81, 117-123):
 * round(clamp(c, 0, 1) * 255), half away from zero, NaN -> 0, for f64
 * canvases (the kernels quantize RT_OUT_U8 frames themselves). */
int rt_canvas_quantize(const double* rgb, uint64_t n_channels, uint8_t* out);

#ifdef __cplusplus
}
#endif

#endif /* RTC_SCENE_H */
