// TypeScript surface of the MI355X drop-in.  Mirrors the reference's Raytracer
// (src/raytracer.ts:33-43, 281-339) and adds FaceEntity (fills src/entities/entity_face.ts).
// Scene types are the reference's own; they are declared structurally here so this package does
// not depend on the reference's sources.

export interface VectorLike { v: number[] }
export interface ColorLike { r: number; g: number; b: number; a: number }
export interface TextureLike { get_color(u: number, v: number): ColorLike; get_size(): [number, number] | undefined }
export interface MaterialLike {
  response_type(point: VectorLike): number;      // ResponseType
  is_mirror(point: VectorLike): boolean;
  is_light_source(): boolean;
  readonly roughness_index: number;
}
export interface SubstanceLike { refractive_index: number }
export interface SkyLike { texture: TextureLike }

/** RaytracerConfig, src/raytracer.ts:33-43 */
export interface RaytracerConfig {
  refmax: number;
  sky: SkyLike;
  default_substance: SubstanceLike | undefined;
  distance_attenuation_factor: number;
}

/** Work counters of a frame (options.stats); without them only frame_ms is set. */
export interface RtStats {
  segments?: number; n_ret?: number; n_slot?: number; n_loc?: number; n_sph?: number; n_box?: number;
  n_tri?: number; n_hit?: number; primary?: number; n_warn?: number; n_fault?: number;
  kernel_ms?: number; frame_ms: number;
}

export interface RaytracerOptions {
  /** HIP device ordinal (default 0) */
  device?: number;
  /** GPUs to split every frame over (row stripes, RCCL gather to devices[0]) */
  devices?: number[];
  /** rows per stripe of the multi-device split (default 8) */
  stripe_rows?: number;
  /** keep per-pixel primary hit entity / node ids and status after each frame */
  keep_ids?: boolean;
  /** fill last_stats with work counters (runs the slower fused counting kernel) */
  stats?: boolean;
  /** 'counter': rough mirrors with the counter-based RNG (include/rt.h RT_SCATTER_COUNTER) */
  scatter?: 'counter';
  /** shadow rays, a build extension the reference lacks (include/rt.h rt_set_lights): at most 4 */
  lights?: PointLight[];
  /** the ambient term of the shadow-ray extension (default 0) */
  ambient?: number;
}

/** A point light of the shadow-ray extension. */
export interface PointLight {
  pos: VectorLike | number[];
  rgb: VectorLike | number[];
}

/** Drop-in for the reference `Raytracer`: same constructor and methods; trace_frame() runs on a GPU. */
export class Raytracer {
  constructor(config: RaytracerConfig, otree: any, camera: any, ebuffer: any, rng: any, options?: RaytracerOptions);
  config: RaytracerConfig;
  set_camera(camera: any): void;
  set_ebuffer(ebuffer: any): void;
  trace_frame(): void;
  readonly tree: any;
  readonly rng: any;
  /** re-flatten the octree before the next frame (after adding or moving entities) */
  invalidate_scene(): void;
  /** release the GPU context */
  close(): void;
  /** shadow rays (build extension): lights and ambient for the next frames; [] turns them off */
  set_lights(lights: PointLight[], ambient?: number): void;
  last_stats: RtStats | null;
  last_hit_entity: Int32Array | null;
  last_hit_node: Int32Array | null;
  last_status: Uint8Array | null;
}

/** The triangle entity (DESIGN.md §Triangle): Entity contract of src/entity.ts:38-101. */
export class FaceEntity {
  constructor(entity_otree: any, material: MaterialLike, texture: TextureLike, substance: SubstanceLike | undefined,
              v0: VectorLike | number[], v1: VectorLike | number[], v2: VectorLike | number[]);
  set_octree(tree: any, flags?: { keep_in_current?: boolean }): void;
  readonly octree: any;
  get_substance(): SubstanceLike | undefined;
  set_substance(s: SubstanceLike | undefined): SubstanceLike | undefined;
  get_vertices(): [VectorLike, VectorLike, VectorLike];
  get_pos(): VectorLike;
  _set_pos(p: VectorLike): VectorLike;
  get_material(): MaterialLike;
  set_material(m: MaterialLike): MaterialLike;
  get_texture(): TextureLike;
  set_texture(t: TextureLike): TextureLike;
  is_within(point: VectorLike): boolean;
  get_aabb(): [VectorLike, number];
  map_uv(p: VectorLike): [number, number];
  collision_info(ray: { get_pos(): VectorLike; get_dir(): VectorLike }):
    { point: VectorLike; material: MaterialLike; texture: TextureLike; normal: VectorLike } | null;
}

export function serialize_scene(otree: any, default_substance?: SubstanceLike): any;
export function camera_desc(camera: any): any;
export function load_addon(): any;
export const RT_ENT_SPHERE: 0;
export const RT_ENT_BOX: 1;
export const RT_ENT_FACE: 2;
