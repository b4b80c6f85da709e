! letkf_core_gpu.f90 — iso_c_binding interface to the MI355X LETKF core (include/cwb_letkf_core.h).
!
! This is the Fortran side of the drop-in boundary: the reference's letkf_driver
! (module_letkf_core.f90:21-298) keeps its variable loop, scatter/gather and tune_q, and
! replaces build_tree + the grid-point loop (:63-64, :209-240) by one call of
! cwbl_analyze_var per variable (INTEGRATION.md shows the edited driver).
!
! Types mirror the C structs field by field (bind(C)); logicals cross as integer(c_int) 0/1.
module letkf_core_gpu
    use iso_c_binding
    implicit none
    private

    integer(c_int), parameter, public :: CWBL_MEM_HOST = 0, CWBL_MEM_DEVICE = 1
    integer(c_int), parameter, public :: CWBL_Q1_REPLICATE = 0, CWBL_Q1_PER_TYPE = 1
    integer,        parameter, public :: CWBL_NUM_GTS_TYPES = 29, CWBL_NUM_RADAR_TYPES = 4

    type, bind(C), public :: cwbl_init_params
        integer(c_int)    :: nmember, device, weight_function
        real(c_float)     :: norain_value
        integer(c_int)    :: q1_mode, reserved
        integer(c_size_t) :: workspace_bytes
    end type cwbl_init_params

    type, bind(C), public :: cwbl_gts_obs          ! type(gts_structure), module_gts_omboma.f90:13-22
        integer(c_int) :: type_id, nvar, nobs, reserved
        type(c_ptr)    :: xyz, obs, error, hdxb, qc
    end type cwbl_gts_obs

    type, bind(C), public :: cwbl_radar_obs        ! type(radar_structure), module_radar.f90:13-16
        integer(c_int) :: type_id, nobs
        type(c_ptr)    :: xyz, obs, hdxb
    end type cwbl_radar_obs

    type, bind(C), public :: cwbl_obs_set
        integer(c_int) :: n_gts, n_radar
        type(c_ptr)    :: gts, radar
        integer(c_int) :: memory, reserved
    end type cwbl_obs_set

    type, bind(C), public :: cwbl_type_params      ! gts_config / radar_variable_config
        integer(c_int) :: use_it, max_lz_pts
        real(c_float)  :: hclr, vclr
        real(c_float)  :: err_muti(5), err_rej(5)
        integer(c_int) :: is_assim(5)
    end type cwbl_type_params

    type, bind(C), public :: cwbl_var_params
        real(c_float)          :: multi_infl
        integer(c_int)         :: use_rtpp
        real(c_float)          :: rtpp_alpha
        integer(c_int)         :: use_rtps
        real(c_float)          :: rtps_alpha
        integer(c_int)         :: tune_q       ! 1: letkf_tune_q after the analysis
        type(cwbl_type_params) :: gts(CWBL_NUM_GTS_TYPES)
        type(cwbl_type_params) :: radar(CWBL_NUM_RADAR_TYPES)
    end type cwbl_var_params

    type, bind(C), public :: cwbl_slab             ! var(nx,ny,nz,0:k-1), module_letkf_core.f90:85
        integer(c_int) :: nx, ny, nz, alt_nx, alt_ny, ix_lim, iy_lim, memory
        type(c_ptr)    :: x, y, alt, var
    end type cwbl_slab

    type, bind(C), public :: cwbl_stats
        integer(c_long_long) :: points, solved, nobs_sum, lz_truncated, nonconverged, &
                                q1_undefined, sweeps_sum
        integer(c_int)       :: max_p, max_sweeps, ntrees, reserved
        real(c_double)       :: ms_total, ms_prep, ms_search, ms_solve, ms_copy
    end type cwbl_stats

    ! projection_nml (module_config.f90:70-75), include/cwb_letkf_ingest.h
    type, bind(C), public :: cwbl_projection
        real(c_float) :: sta_lon, cen_lat, truelat1, truelat2
    end type cwbl_projection

    public :: cwbl_init, cwbl_set_obs, cwbl_analyze_var, cwbl_solve_batch, cwbl_search, &
              cwbl_pack_columns, cwbl_unpack_columns, cwbl_pack_members, cwbl_unpack_members, &
              cwbl_vcoord_mean, &
              cwbl_member_sum, cwbl_scale, cwbl_set_stream, cwbl_set_option, &
              cwbl_finalize, cwbl_abi_version, cwbl_error, cwbl_check
    ! host obs ingest (include/cwb_letkf_ingest.h); file names and varname are passed as
    ! trim(name)//c_null_char
    public :: cwbl_lonlat_to_xy, cwbl_ingest_create, cwbl_ingest_destroy, cwbl_ingest_read_gts, &
              cwbl_ingest_read_radar, cwbl_ingest_obs_set, cwbl_ingest_type_meta, &
              cwbl_ingest_wire_words, cwbl_ingest_pack_wire

    interface
        integer(c_int) function cwbl_init(p) bind(C, name='cwbl_init')
            import :: c_int, cwbl_init_params
            type(cwbl_init_params), intent(in) :: p
        end function cwbl_init

        integer(c_int) function cwbl_set_obs(o) bind(C, name='cwbl_set_obs')
            import :: c_int, cwbl_obs_set
            type(cwbl_obs_set), intent(in) :: o
        end function cwbl_set_obs

        integer(c_int) function cwbl_analyze_var(vp, slab, stats) bind(C, name='cwbl_analyze_var')
            import :: c_int, cwbl_var_params, cwbl_slab, cwbl_stats
            type(cwbl_var_params), intent(in)    :: vp
            type(cwbl_slab),       intent(in)    :: slab
            type(cwbl_stats),      intent(inout) :: stats
        end function cwbl_analyze_var

        integer(c_int) function cwbl_solve_batch(npts, col_off, yo, yb, xb, inflat, use_rtpp, &
                rtpp_alpha, use_rtps, rtps_alpha, xa, evals, memory) bind(C, name='cwbl_solve_batch')
            import :: c_int, c_float, c_ptr
            integer(c_int), value :: npts, use_rtpp, use_rtps, memory
            real(c_float),  value :: inflat, rtpp_alpha, rtps_alpha
            type(c_ptr),    value :: col_off, yo, yb, xb, xa, evals
        end function cwbl_solve_batch

        integer(c_int) function cwbl_search(nobs, obs_xyz, hclr, vclr, max_lz_pts, nq, q_xyz, &
                nfound, idx, r2, memory) bind(C, name='cwbl_search')
            import :: c_int, c_float, c_ptr
            integer(c_int), value :: nobs, max_lz_pts, nq, memory
            real(c_float),  value :: hclr, vclr
            type(c_ptr),    value :: obs_xyz, q_xyz, nfound, idx, r2
        end function cwbl_search

        ! member <-> column transposes (module_mpi_util.f90:190-358, 445-580); device pointers
        integer(c_int) function cwbl_pack_columns(global, nx, ny, nz, px, py, send) &
                bind(C, name='cwbl_pack_columns')
            import :: c_int, c_ptr
            type(c_ptr),    value :: global, send
            integer(c_int), value :: nx, ny, nz, px, py
        end function cwbl_pack_columns

        integer(c_int) function cwbl_unpack_columns(recv, nx, ny, nz, px, py, global) &
                bind(C, name='cwbl_unpack_columns')
            import :: c_int, c_ptr
            type(c_ptr),    value :: recv, global
            integer(c_int), value :: nx, ny, nz, px, py
        end function cwbl_unpack_columns

        integer(c_int) function cwbl_pack_members(global, gstride, nm, nx, ny, nz, px, py, &
                send, sstride) bind(C, name='cwbl_pack_members')
            import :: c_int, c_long_long, c_ptr
            type(c_ptr),          value :: global, send
            integer(c_long_long), value :: gstride, sstride
            integer(c_int),       value :: nm, nx, ny, nz, px, py
        end function cwbl_pack_members

        integer(c_int) function cwbl_unpack_members(recv, rstride, nm, nx, ny, nz, px, py, &
                global, gstride) bind(C, name='cwbl_unpack_members')
            import :: c_int, c_long_long, c_ptr
            type(c_ptr),          value :: recv, global
            integer(c_long_long), value :: rstride, gstride
            integer(c_int),       value :: nm, nx, ny, nz, px, py
        end function cwbl_unpack_members

        integer(c_int) function cwbl_vcoord_mean(ph, n2d, nz_ph, k, stagger, g, alt) &
                bind(C, name='cwbl_vcoord_mean')
            import :: c_int, c_long_long, c_float, c_ptr
            type(c_ptr),          value :: ph, alt
            integer(c_long_long), value :: n2d
            integer(c_int),       value :: nz_ph, k, stagger
            real(c_float),        value :: g
        end function cwbl_vcoord_mean

        ! write_mean (module_grid.f90:744-840): member sum of device fields(n, nm), member
        ! slowest, and sscal; the cross-rank sum between the two is one reduce (MPI or RCCL)
        integer(c_int) function cwbl_member_sum(fields, n, nm, out) bind(C, name='cwbl_member_sum')
            import :: c_int, c_long_long, c_ptr
            type(c_ptr),          value :: fields, out
            integer(c_long_long), value :: n
            integer(c_int),       value :: nm
        end function cwbl_member_sum

        integer(c_int) function cwbl_scale(x, n, alpha) bind(C, name='cwbl_scale')
            import :: c_int, c_long_long, c_float, c_ptr
            type(c_ptr),          value :: x
            integer(c_long_long), value :: n
            real(c_float),        value :: alpha
        end function cwbl_scale

        ! HIP stream (hipStream_t, c_null_ptr = the null stream) whose queued work device
        ! pointers handed to the library may still depend on
        integer(c_int) function cwbl_set_stream(stream) bind(C, name='cwbl_set_stream')
            import :: c_int, c_ptr
            type(c_ptr), value :: stream
        end function cwbl_set_stream

        ! proj_type%init + %lonlat_to_xy (module_projection.f90:21-50) for n points
        integer(c_int) function cwbl_lonlat_to_xy(proj, n, lon, lat, x, y) &
                bind(C, name='cwbl_lonlat_to_xy')
            import :: c_int, c_long_long, c_float, cwbl_projection
            type(cwbl_projection), intent(in)  :: proj
            integer(c_long_long),  value       :: n
            real(c_float),         intent(in)  :: lon(*), lat(*)
            real(c_float),         intent(out) :: x(*), y(*)
        end function cwbl_lonlat_to_xy

        type(c_ptr) function cwbl_ingest_create(nmember, proj) bind(C, name='cwbl_ingest_create')
            import :: c_ptr, c_int, cwbl_projection
            integer(c_int), value             :: nmember
            type(cwbl_projection), intent(in) :: proj
        end function cwbl_ingest_create

        subroutine cwbl_ingest_destroy(h) bind(C, name='cwbl_ingest_destroy')
            import :: c_ptr
            type(c_ptr), value :: h
        end subroutine cwbl_ingest_destroy

        ! read_gts_omboma (module_gts_omboma.f90:48-506) of one member; member -1: from the name
        integer(c_int) function cwbl_ingest_read_gts(h, member, gts_file, obs_gts_file) &
                bind(C, name='cwbl_ingest_read_gts')
            import :: c_int, c_ptr, c_char
            type(c_ptr),    value :: h
            integer(c_int), value :: member
            character(kind=c_char), intent(in) :: gts_file(*), obs_gts_file(*)
        end function cwbl_ingest_read_gts

        ! read_radar (module_radar.f90:30-118); varname 'MR', 'VR', 'MD' or 'MK'
        integer(c_int) function cwbl_ingest_read_radar(h, member, file, varname) &
                bind(C, name='cwbl_ingest_read_radar')
            import :: c_int, c_ptr, c_char
            type(c_ptr),    value :: h
            integer(c_int), value :: member
            character(kind=c_char), intent(in) :: file(*), varname(*)
        end function cwbl_ingest_read_radar

        ! the set read so far as a host-memory cwbl_obs_set (views into the handle)
        integer(c_int) function cwbl_ingest_obs_set(h, os) bind(C, name='cwbl_ingest_obs_set')
            import :: c_int, c_ptr, cwbl_obs_set
            type(c_ptr), value                :: h
            type(cwbl_obs_set), intent(out)   :: os
        end function cwbl_ingest_obs_set

        integer(c_int) function cwbl_ingest_type_meta(h, family, type_id, nvar, nobs, ids, lat, &
                lon, alt) bind(C, name='cwbl_ingest_type_meta')
            import :: c_int, c_ptr
            type(c_ptr),    value         :: h
            integer(c_int), value         :: family, type_id
            integer(c_int), intent(out)   :: nvar, nobs
            type(c_ptr),    intent(out)   :: ids, lat, lon, alt
        end function cwbl_ingest_type_meta

        ! the one-buffer wire format replacing gts_distribute / radar_distribute
        ! (module_gts_omboma.f90:508-611, module_radar.f90:120-186): one MPI_Bcast of
        ! cwbl_ingest_wire_words(h) reals from the reading rank
        integer(c_long_long) function cwbl_ingest_wire_words(h) bind(C, name='cwbl_ingest_wire_words')
            import :: c_long_long, c_ptr
            type(c_ptr), value :: h
        end function cwbl_ingest_wire_words

        integer(c_int) function cwbl_ingest_pack_wire(h, buf, cap_words) &
                bind(C, name='cwbl_ingest_pack_wire')
            import :: c_int, c_long_long, c_float, c_ptr
            type(c_ptr),          value       :: h
            real(c_float),        intent(out) :: buf(*)
            integer(c_long_long), value       :: cap_words
        end function cwbl_ingest_pack_wire

        ! path options (A/B measurement; include/cwb_letkf_core.h CWBL_OPT_*), after cwbl_init
        integer(c_int) function cwbl_set_option(option, val) bind(C, name='cwbl_set_option')
            import :: c_int, c_long_long
            integer(c_int),       value :: option
            integer(c_long_long), value :: val
        end function cwbl_set_option

        integer(c_int) function cwbl_finalize() bind(C, name='cwbl_finalize')
            import :: c_int
        end function cwbl_finalize

        integer(c_int) function cwbl_abi_version() bind(C, name='cwbl_abi_version')
            import :: c_int
        end function cwbl_abi_version

        type(c_ptr) function cwbl_last_error_c() bind(C, name='cwbl_last_error')
            import :: c_ptr
        end function cwbl_last_error_c
    end interface

contains

    ! cwbl_last_error() as a Fortran string
    function cwbl_error() result(msg)
        character(len=:), allocatable :: msg
        type(c_ptr) :: p
        character(kind=c_char), pointer :: s(:)
        integer :: n
        p = cwbl_last_error_c()
        msg = ''
        if (.not. c_associated(p)) return
        call c_f_pointer(p, s, [4096])
        n = 0
        do while (n < 4096)
            if (s(n+1) == c_null_char) exit
            n = n + 1
        end do
        allocate(character(len=n) :: msg)
        msg = transfer(s(1:n), msg)
    end function cwbl_error

    ! The reference's error convention: a failing call ends the program with `stop "<msg>"`
    ! (module_config.f90:123-146, module_netcdf_io.f90:378-386).  The library itself never exits.
    subroutine cwbl_check(rc, what)
        integer(c_int),   intent(in) :: rc
        character(len=*), intent(in) :: what
        if (rc /= 0) then
            print '(a,a,i0,a,a)', what, ' failed, code ', rc, ': ', cwbl_error()
            stop "LETKF core error"
        end if
    end subroutine cwbl_check

end module letkf_core_gpu
