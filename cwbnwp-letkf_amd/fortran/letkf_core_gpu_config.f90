! letkf_core_gpu_config.f90 — fills the ABI's per-variable parameter block from the
! reference's namelist state (module config, module_config.f90:1-150).
!
! Compiled against the reference's own `config`/`param` modules (it is part of the Fortran
! host, which keeps read_namelist and input.nml as the configuration surface).  The order of
! the per-obs-variable entries is the order letkf_yoyb builds is_assim/err_muti/err_rej
! (module_letkf_core.f90:349-417).
module letkf_core_gpu_config
    use iso_c_binding
    use letkf_core_gpu
    use config
    use param, only : sound, synop, gpspw, metar, ships, dbz, vr, zdr, kdp
    implicit none
    private
    public :: var_params_from_namelist, init_params_from_namelist

contains

    subroutine init_params_from_namelist(device, p)
        integer,                intent(in)  :: device
        type(cwbl_init_params), intent(out) :: p
        p%nmember         = nmember
        p%device          = device
        p%weight_function = weight_function
        p%norain_value    = norain_value
        p%q1_mode         = CWBL_Q1_REPLICATE
        p%reserved        = 0
        p%workspace_bytes = 0
    end subroutine init_params_from_namelist

    subroutine var_params_from_namelist(ivar, vp)
        integer,               intent(in)  :: ivar
        type(cwbl_var_params), intent(out) :: vp
        integer :: i
        vp%multi_infl = multi_infl(ivar)
        vp%use_rtpp   = merge(1, 0, use_RTPP(ivar))
        vp%rtpp_alpha = RTPP_Alpha(ivar)
        vp%use_rtps   = merge(1, 0, use_RTPS(ivar))
        vp%rtps_alpha = RTPS_Alpha(ivar)
        ! letkf_driver tunes the hydrometeor species after the loop (:253-278)
        select case (trim(var_update(ivar)))
        case ('QVAPOR', 'QRAIN', 'QSNOW', 'QGRAUP', 'QHAIL', 'QNRAIN', 'QNSNOW', &
              'QNGRAUPEL', 'QNHAIL')
            vp%tune_q = 1
        case default
            vp%tune_q = 0
        end select
        do i = 1, CWBL_NUM_GTS_TYPES
            call off(vp%gts(i))
        end do
        do i = 1, CWBL_NUM_RADAR_TYPES
            call off(vp%radar(i))
        end do
        call gts5(synop_nml, vp%gts(synop))
        call gts5(metar_nml, vp%gts(metar))
        call gts5(ships_nml, vp%gts(ships))
        call gts_common(sound_nml, vp%gts(sound))
        call put(vp%gts(sound), 1, sound_nml%u)
        call put(vp%gts(sound), 2, sound_nml%v)
        call put(vp%gts(sound), 3, sound_nml%t)
        call put(vp%gts(sound), 4, sound_nml%q)
        call gts_common(gpspw_nml, vp%gts(gpspw))
        call put(vp%gts(gpspw), 1, gpspw_nml%tpw)
        call radar1(radar_nml%dbz, vp%radar(dbz))
        call radar1(radar_nml%vr,  vp%radar(vr))
        call radar1(radar_nml%zdr, vp%radar(zdr))
        call radar1(radar_nml%kdp, vp%radar(kdp))
    contains
        subroutine off(t)
            type(cwbl_type_params), intent(out) :: t
            t%use_it = 0; t%max_lz_pts = 0; t%hclr = -1.; t%vclr = -1.
            t%err_muti = 1.; t%err_rej = 5.; t%is_assim = 0
        end subroutine off
        subroutine gts_common(c, t)
            type(gts_config),       intent(in)    :: c
            type(cwbl_type_params), intent(inout) :: t
            t%use_it     = merge(1, 0, c%use_it)
            t%max_lz_pts = c%max_lz_pts
            t%hclr       = c%hclr(ivar)
            t%vclr       = c%vclr(ivar)
        end subroutine gts_common
        subroutine put(t, k, v)
            type(cwbl_type_params),    intent(inout) :: t
            integer,                   intent(in)    :: k
            type(gts_variable_config), intent(in)    :: v
            t%err_muti(k) = v%err_muti
            t%err_rej(k)  = v%err_rej
            t%is_assim(k) = merge(1, 0, v%is_assim(ivar))
        end subroutine put
        subroutine gts5(c, t)
            type(gts_config),       intent(in)    :: c
            type(cwbl_type_params), intent(inout) :: t
            call gts_common(c, t)
            call put(t, 1, c%u)
            call put(t, 2, c%v)
            call put(t, 3, c%t)
            call put(t, 4, c%p)
            call put(t, 5, c%q)
        end subroutine gts5
        subroutine radar1(c, t)
            type(radar_variable_config), intent(in)    :: c
            type(cwbl_type_params),      intent(inout) :: t
            t%use_it      = merge(1, 0, c%use_it)
            t%max_lz_pts  = c%max_lz_pts
            t%hclr        = c%hclr(ivar)
            t%vclr        = c%vclr(ivar)
            t%err_muti(1) = c%error
            t%err_rej(1)  = c%err_rej
        end subroutine radar1
    end subroutine var_params_from_namelist

end module letkf_core_gpu_config
