//! massrt-sys: the reference's side of the drop-in boundary.
//!
//! The reference renders a frame with
//! `render(image, event_proxy, world, camera, frame_limit)` (src/main.rs:150-156,
//! called by `worker`, main.rs:114-118). With this crate that function keeps its
//! signature and body shape: the world is flattened once through `SceneSink`
//! (each reference type implements `Export`), uploaded,
//! and `render()` below runs the reference's pass loop over a device-resident
//! `GpuImage` (one context may span several GPUs), handing the sums and the
//! pass count to the caller's `Image` after every batch.
//!
//! Source only here (no Rust toolchain in the build image); the FFI layout is
//! checked against include/massrt.h by tests/test_rust_binding.py.

pub mod sys;

use std::collections::HashMap;
use std::ffi::{CStr, CString};
use sys::*;

/// Error of a massrt call: the status code and `mrt_last_error` text.
#[derive(Debug, Clone)]
pub struct MrtError {
    pub code: i32,
    pub message: String,
}

/// Implemented by the reference's `Intersect` types (geom.rs) so that
/// `Box<dyn Intersect>` can cross the FFI: returns the child reference
/// `mrt_ref(kind, index)` of the exported object.
pub trait Export {
    fn export(&self, sink: &mut SceneSink) -> u32;
}

/// Flat scene under construction (the reference tree as built: node for node).
#[derive(Default)]
pub struct SceneSink {
    pub nodes: Vec<mrt_node>,
    pub spheres: Vec<mrt_sphere>,
    pub triangles: Vec<mrt_triangle>,
    pub instances: Vec<mrt_instance>,
    pub models: Vec<mrt_model>,
    pub materials: Vec<mrt_material>,
    pub surfaces: Vec<mrt_surface>,
    pub textures: Vec<mrt_texture>,
    pub volumes: Vec<mrt_volume>,
    /// RGBA8 storage the `textures` entries point into (kept alive by the sink)
    pub texels: Vec<Vec<u8>>,
    /// shared BLAS (Arc<BvhNode>) exported once, keyed by Arc::as_ptr
    pub blas: HashMap<usize, u32>,
    /// materials / surfaces interned by the address of the Arc they came from
    pub material_ids: HashMap<usize, u32>,
    pub surface_ids: HashMap<usize, u32>,
}

impl SceneSink {
    pub fn push_node(&mut self) -> usize {
        self.nodes.push(mrt_node::default());
        self.nodes.len() - 1
    }

    /// BLAS root node of a shared tree, exporting it on first use.
    pub fn blas_root<T: Export + ?Sized>(&mut self, key: usize, tree: &T) -> u32 {
        if let Some(&r) = self.blas.get(&key) {
            return r;
        }
        let r = tree.export(self) & 0x0FFF_FFFF;
        self.blas.insert(key, r);
        r
    }

    pub fn texture(&mut self, width: u32, height: u32, wrap: u32, rgba: Vec<u8>) -> u32 {
        assert_eq!(rgba.len(), (width * height * 4) as usize);
        self.textures.push(mrt_texture { width, height, wrap, rgba: rgba.as_ptr() });
        self.texels.push(rgba); // the Vec's heap buffer does not move
        (self.textures.len() - 1) as u32
    }

    /// The boundary description; borrows the sink (valid while it lives).
    pub fn desc(&self, roots: &[u32], background: mrt_background) -> mrt_scene_desc {
        mrt_scene_desc {
            nodes: self.nodes.as_ptr(),
            n_nodes: self.nodes.len() as u32,
            roots: roots.as_ptr(),
            n_roots: roots.len() as u32,
            spheres: self.spheres.as_ptr(),
            n_spheres: self.spheres.len() as u32,
            triangles: self.triangles.as_ptr(),
            n_triangles: self.triangles.len() as u32,
            instances: self.instances.as_ptr(),
            n_instances: self.instances.len() as u32,
            models: self.models.as_ptr(),
            n_models: self.models.len() as u32,
            materials: self.materials.as_ptr(),
            n_materials: self.materials.len() as u32,
            surfaces: self.surfaces.as_ptr(),
            n_surfaces: self.surfaces.len() as u32,
            textures: self.textures.as_ptr(),
            n_textures: self.textures.len() as u32,
            background,
            volumes: self.volumes.as_ptr(),
            n_volumes: self.volumes.len() as u32,
        }
    }
}

/// One GPU context (mrt_ctx); destroyed on drop.
pub struct Context {
    raw: *mut mrt_ctx,
}

unsafe impl Send for Context {}

impl Context {
    /// One context over several devices (mrt_create_multi): each renders its
    /// share of the frame's tiles; reads gather them.
    pub fn new_multi(devices: &[i32]) -> Result<Context, MrtError> {
        let mut raw = std::ptr::null_mut();
        let rc = unsafe { mrt_create_multi(devices.len() as i32, devices.as_ptr(), &mut raw) };
        if rc != MRT_OK {
            let message = unsafe { CStr::from_ptr(mrt_global_last_error()) }.to_string_lossy().into_owned();
            return Err(MrtError { code: rc, message });
        }
        Ok(Context { raw })
    }

    pub fn devices(&self) -> Result<Vec<i32>, MrtError> {
        let mut n = 0i32;
        self.check(unsafe { mrt_context_devices(self.raw, &mut n, std::ptr::null_mut()) })?;
        let mut ids = vec![0i32; n as usize];
        self.check(unsafe { mrt_context_devices(self.raw, &mut n, ids.as_mut_ptr()) })?;
        Ok(ids)
    }

    pub fn new(device: i32) -> Result<Context, MrtError> {
        let mut raw = std::ptr::null_mut();
        let rc = unsafe { mrt_create(device, &mut raw) };
        if rc != MRT_OK {
            let message = unsafe { CStr::from_ptr(mrt_global_last_error()) }.to_string_lossy().into_owned();
            return Err(MrtError { code: rc, message });
        }
        Ok(Context { raw })
    }

    pub fn check(&self, rc: i32) -> Result<(), MrtError> {
        if rc == MRT_OK {
            return Ok(());
        }
        let message = unsafe { CStr::from_ptr(mrt_last_error(self.raw)) }.to_string_lossy().into_owned();
        Err(MrtError { code: rc, message })
    }

    pub fn upload(&mut self, scene: &mrt_scene_desc, camera: &mrt_camera) -> Result<(), MrtError> {
        self.check(unsafe { mrt_upload_scene(self.raw, scene) })?;
        self.check(unsafe { mrt_set_camera(self.raw, camera) })
    }

    /// Samples [spp_begin, spp_begin + spp_count) of every pixel (of this
    /// shard) ADDED into `rgb` (w*h*3) and `bounces` (w*h), y = 0 the bottom row.
    pub fn render(&mut self, args: &mrt_render_args, rgb: &mut [f32], bounces: &mut [u32]) -> Result<(), MrtError> {
        let n = (args.width * args.height) as usize;
        assert!(rgb.len() >= 3 * n && bounces.len() >= n);
        self.check(unsafe { mrt_render(self.raw, args, rgb.as_mut_ptr(), bounces.as_mut_ptr()) })
    }

    pub fn prepass(&mut self, w: u32, h: u32, seed: u64, albedo: &mut [f32], normal: &mut [f32])
        -> Result<(), MrtError> {
        let n = (w * h * 3) as usize;
        assert!(albedo.len() >= n && normal.len() >= n);
        self.check(unsafe { mrt_prepass(self.raw, w, h, seed, albedo.as_mut_ptr(), normal.as_mut_ptr()) })
    }

    pub fn tonemap(&mut self, w: u32, h: u32, rgb: &[f32], bounces: &[u32], passes: u32, mode: u32,
                   out: &mut [u8]) -> Result<(), MrtError> {
        assert!(out.len() >= (w * h * 3) as usize);
        self.check(unsafe { mrt_tonemap(self.raw, w, h, rgb.as_ptr(), bounces.as_ptr(), passes, mode, out.as_mut_ptr()) })
    }

    /// A tuning option of the context (mrt_set_option; names in massrt.h).
    pub fn set_option(&mut self, name: &str, value: i64) -> Result<(), MrtError> {
        let c = CString::new(name).expect("option name without NUL");
        self.check(unsafe { mrt_set_option(self.raw, c.as_ptr(), value) })
    }

    /// The gather transport of a multi-device context ("rccl", "peer", ...).
    pub fn transport(&self) -> String {
        unsafe { CStr::from_ptr(mrt_context_transport(self.raw)) }.to_string_lossy().into_owned()
    }

    pub fn raw(&self) -> *mut mrt_ctx {
        self.raw
    }
}

impl Drop for Context {
    fn drop(&mut self) {
        unsafe {
            mrt_destroy(self.raw);
        }
    }
}

/// The reference's `Image` (main.rs:598-638) kept in HBM: colour sums, depth
/// sums and the pass count live on the context's device(s) (`mrt_image`);
/// passes add to it without a host round trip and only `read` / `tonemap`
/// cross PCIe. On a multi-device context every device keeps its own tiles
/// and a read gathers them (RCCL over xGMI).
pub struct GpuImage<'a> {
    raw: *mut mrt_image,
    ctx: &'a Context,
    pub width: u32,
    pub height: u32,
}

impl<'a> GpuImage<'a> {
    pub fn new(ctx: &'a Context, width: u32, height: u32) -> Result<GpuImage<'a>, MrtError> {
        let mut raw = std::ptr::null_mut();
        ctx.check(unsafe { mrt_image_create(ctx.raw, width, height, &mut raw) })?;
        Ok(GpuImage { raw, ctx, width, height })
    }

    /// Image::clear (main.rs:749-758)
    pub fn clear(&mut self) -> Result<(), MrtError> {
        self.ctx.check(unsafe { mrt_image_clear(self.raw) })
    }

    /// `passes` 1-spp passes merged (Image::merge x passes): samples
    /// [spp_begin, spp_begin + passes) of every pixel under `seed`.
    pub fn render(&mut self, seed: u64, spp_begin: u32, passes: u32, max_depth: u32) -> Result<(), MrtError> {
        self.ctx.check(unsafe { mrt_image_render(self.raw, seed, spp_begin, passes, max_depth, 0) })
    }

    /// Camera::albedo_normal pre-pass into the image (main.rs:162-222)
    pub fn prepass(&mut self, seed: u64) -> Result<(), MrtError> {
        self.ctx.check(unsafe { mrt_image_prepass(self.raw, seed) })
    }

    /// Sums (w*h*3), depths (w*h); returns the pass count (Image::pixels.0).
    pub fn read(&mut self, rgb: &mut [f32], bounces: &mut [u32]) -> Result<u32, MrtError> {
        let n = (self.width * self.height) as usize;
        assert!(rgb.len() >= 3 * n && bounces.len() >= n);
        let mut passes = 0u32;
        self.ctx.check(unsafe { mrt_image_read(self.raw, rgb.as_mut_ptr(), bounces.as_mut_ptr(), &mut passes) })?;
        Ok(passes)
    }

    pub fn passes(&mut self) -> Result<u32, MrtError> {
        let mut passes = 0u32;
        self.ctx.check(unsafe { mrt_image_read(self.raw, std::ptr::null_mut(), std::ptr::null_mut(), &mut passes) })?;
        Ok(passes)
    }

    /// Image::to_rgb_bytes + dump's row flip (main.rs:640-722, 763-766): w*h*3 bytes.
    pub fn tonemap(&mut self, mode: u32, out: &mut [u8]) -> Result<(), MrtError> {
        assert!(out.len() >= (self.width * self.height * 3) as usize);
        self.ctx.check(unsafe { mrt_image_tonemap(self.raw, mode, out.as_mut_ptr()) })
    }
}

impl<'a> Drop for GpuImage<'a> {
    fn drop(&mut self) {
        unsafe {
            mrt_image_destroy(self.raw);
        }
    }
}

/// Where a frame's samples come from. The reference's render threads draw
/// from thread-local fastrand streams seeded afresh for every render() call
/// (main.rs:167-250), so no two frames share samples. Here sample s of pixel
/// p is keyed (seed, p, s); the sample index keeps counting across frames,
/// and the seed moves on when it would wrap.
#[derive(Debug, Clone, Copy)]
pub struct SampleStreams {
    pub seed: u64,
    pub next_sample: u32,
}

impl SampleStreams {
    pub fn new(seed: u64) -> SampleStreams {
        SampleStreams { seed, next_sample: 0 }
    }

    /// The (seed, first sample) of the next `n` consecutive samples.
    pub fn take(&mut self, n: u32) -> (u64, u32) {
        if self.next_sample as u64 + n as u64 > u32::MAX as u64 {
            self.seed = self.seed.wrapping_add(1);
            self.next_sample = 0;
        }
        let first = self.next_sample;
        self.next_sample += n;
        (self.seed, first)
    }
}

/// render()'s worker count: num_cpus - 2, at least 1 (main.rs:159-160).
pub fn default_workers() -> u32 {
    let cpus = std::thread::available_parallelism().map(|n| n.get() as i64).unwrap_or(1);
    (cpus - 2).max(1) as u32
}

pub struct RenderOptions {
    pub max_depth: u32,
    /// the reference's render thread count; `frame_limit` counts passes per worker
    pub workers: u32,
    /// 1-spp passes per GPU call (one `update` per batch). The default 256
    /// covers a frame's passes up to 256 workers in one call, so the UI sees
    /// one update per frame as in main.rs:274-278; bigger calls also keep the
    /// per-call drain tail small
    pub batch: u32,
    pub prepass: bool,
}

impl Default for RenderOptions {
    fn default() -> RenderOptions {
        RenderOptions { max_depth: 50, workers: default_workers(), batch: 256, prepass: true }
    }
}

/// render(image, event_proxy, world, camera, frame_limit) (main.rs:150-295)
/// over the GPU, with the reference's accounting:
///  * the albedo/normal pre-pass first (main.rs:162-222), then Image::clear
///    (main.rs:233);
///  * each of `workers` threads renders `frame_limit` whole 1-spp passes
///    (None: until `keep_going` says stop) and each pass is one merge, so a
///    frame gets workers * frame_limit passes (main.rs:243-280);
///  * the passes run `batch` at a time in one mrt_image_render call, and
///    `update` (the reference's UserEvent::Update, main.rs:274-278) sees the
///    image after each batch with its pass count;
///  * `keep_going` is checked before each batch (QUICK_PASS, main.rs:224-231,
///    282-284).
/// Returns the passes rendered.
pub fn render<U, K>(image: &mut GpuImage, streams: &mut SampleStreams, frame_limit: Option<u32>,
                    opts: &RenderOptions, mut update: U, mut keep_going: K) -> Result<u64, MrtError>
where
    U: FnMut(&mut GpuImage, u32) -> Result<(), MrtError>,
    K: FnMut() -> bool,
{
    if opts.prepass {
        image.prepass(streams.seed)?;
    }
    image.clear()?;
    let total = frame_limit.map(|f| f as u64 * opts.workers.max(1) as u64);
    let batch = opts.batch.max(1) as u64;
    let mut done = 0u64;
    while total.map_or(true, |t| done < t) {
        if !keep_going() {
            break;
        }
        let k = total.map_or(batch, |t| (t - done).min(batch)) as u32;
        let (seed, first) = streams.take(k);
        image.render(seed, first, k, opts.max_depth)?;
        done += k as u64;
        let passes = image.passes()?;
        update(image, passes)?;
    }
    Ok(done)
}
