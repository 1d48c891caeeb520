//! massrt-sys: the reference's side of the drop-in boundary.
//!
//! The reference renders a frame with
//! `render(image, event_proxy, world, camera, frame_limit)` (src/main.rs:150-156,
//! called by `worker`, main.rs:114-118). With this crate that function keeps its
//! signature and body shape: the world is flattened once through `SceneSink`
//! (each reference type implements `Export`), uploaded,
//! and every pass is one `mrt_render` call whose sums are merged into the
//! shared `Image` exactly like `Image::merge` (main.rs:629-638).
//!
//! Source only here (no Rust toolchain in the build image); the FFI layout is
//! checked against include/massrt.h by tests/test_rust_binding.py.

pub mod sys;

use std::collections::HashMap;
use std::ffi::CStr;
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
    pub fn new(device: i32) -> Result<Context, MrtError> {
        let mut raw = std::ptr::null_mut();
        let rc = unsafe { mrt_create(device, &mut raw) };
        if rc != MRT_OK {
            let message = unsafe { CStr::from_ptr(mrt_global_last_error()) }.to_string_lossy().into_owned();
            return Err(MrtError { code: rc, message });
        }
        Ok(Context { raw })
    }

    fn check(&self, rc: i32) -> Result<(), MrtError> {
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

/// render()'s pass loop over the GPU (main.rs:235-290): `frame_limit` passes
/// of 1 spp each (None = until `keep_going` says stop); after each pass the
/// accumulated sums and the pass count go to `merge` (Image::merge).
pub fn render_passes<F, K>(ctx: &mut Context, width: u32, height: u32, max_depth: u32, frame_limit: Option<u32>,
                           mut merge: F, mut keep_going: K) -> Result<(), MrtError>
where
    F: FnMut(&[f32], &[u32], u32),
    K: FnMut() -> bool,
{
    let n = (width * height) as usize;
    let mut rgb = vec![0f32; 3 * n];
    let mut bounces = vec![0u32; n];
    let mut pass = 0u32;
    while frame_limit.map_or(true, |limit| pass < limit) && keep_going() {
        let args = mrt_render_args { width, height, spp_begin: pass, spp_count: 1, seed: 1, max_depth,
                                     shard_index: 0, shard_count: 1, flags: 0 };
        ctx.render(&args, &mut rgb, &mut bounces)?;
        pass += 1;
        merge(&rgb, &bounces, pass);
    }
    Ok(())
}
