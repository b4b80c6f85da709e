! ref_harness.f90 — drives the reference's own compiled code to produce golden vectors.
!
! TEST INFRASTRUCTURE ONLY (built by oracle/ref/build_ref.sh into oracle/_ref/).
! Real reference code exercised: module param / config (read_namelist) / eigen
! (set_optimal_workspace_for_eigen, inverse_matrix, sqrt_matrix) / kdtree2_module
! (kdtree2_create, kdtree2_r_nearest) and the source text of letkf_solve, letkf_tune_q and
! Gaspari_Cohn_1999.  The glue that the reference keeps in modules we cannot compile here
! (build_tree/get_lz normalisation, letkf_yoyb, the driver loop) is restated below,
! line for line, with the file:line it follows.
!
! Usage: ref_harness <mode> <in.bin> <out.bin>,
! modes: consts | solve | search | gc | driver | tuneq
! All files are unformatted stream (little-endian int32 / real32 / real64).
module harness_lib
    use param
    use config
    use eigen
    use kdtree2_module
    use ref_extract
    implicit none

    character(len=512) :: fin, fout

contains

    ! read_namelist (module_config.f90:328-397) with nmember = k (plus any extra namelist
    ! lines per group), then the set-up calls of cwb_letkf.f90:37-38.
    subroutine setup_k(k, ctl, obsl, infl)
        integer, intent(in)                    :: k
        character(len=*), intent(in), optional :: ctl, obsl, infl
        character(len=600)  :: nmlfile
        nmlfile = trim(fout)//'.nml'
        open(31, file=trim(nmlfile), status='replace', action='write')
        write(31, '(a)') '&control'
        write(31, '(a,i0)') ' nmember = ', k
        if (present(ctl)) write(31, '(a)') ctl
        write(31, '(a)') '/'
        write(31, '(a)') '&projection'
        write(31, '(a)') '/'
        write(31, '(a)') '&observations'
        if (present(obsl)) write(31, '(a)') obsl
        write(31, '(a)') '/'
        write(31, '(a)') '&inflation'
        if (present(infl)) write(31, '(a)') infl
        write(31, '(a)') '/'
        close(31)
        call read_namelist(trim(nmlfile))
        open(31, file=trim(nmlfile), status='old')
        close(31, status='delete')
        call set_optimal_workspace_for_eigen(nmember)
        call set_ensemble_constants(nmember)
    end subroutine setup_k

    subroutine do_consts
        real, parameter :: r2 = gc1999 * gc1999          ! module_localization.f90:202
        call setup_k(8)
        open(21, file=trim(fout), access='stream', form='unformatted', status='replace')
        write(21) gc1999, r2, nmember_inv, nmember_1_inv
        close(21)
    end subroutine do_consts

    ! letkf_solve KATs.  in: k npts use_rtpp use_rtps (i4) multi_infl rtpp_a rtps_a (r4),
    ! then per point p (i4) xb(k) yo(p) yb(k,p) (r4).  out: per point xa(k) (r4), lam(k) (r8)
    subroutine do_solve
        integer :: k, npts, irtpp, irtps, ip, p, info
        real    :: multi_infl, rtpp_a, rtps_a, inflat
        real,   allocatable :: xb(:), yo(:), yb(:,:), xa(:)
        real*8, allocatable :: amat(:,:), yb8(:,:), lam(:)
        integer :: i
        open(40, file=trim(fin), access='stream', form='unformatted', status='old')
        read(40) k, npts, irtpp, irtps
        read(40) multi_infl, rtpp_a, rtps_a
        call setup_k(k)
        inflat = (nmember-1) / multi_infl                    ! module_letkf_core.f90:68
        open(21, file=trim(fout), access='stream', form='unformatted', status='replace')
        allocate(xb(k), xa(k), amat(k,k), lam(k))
        do ip = 1, npts
            read(40) p
            allocate(yo(p), yb(k,p), yb8(k,p))
            read(40) xb, yo, yb
            ! eigenvalues as inverse_matrix obtains them (module_eigen.f90:48-49) from the
            ! matrix letkf_solve forms (module_letkf_core.f90:628-649)
            yb8 = dble(yb)
            amat = 0d0
            do i = 1, k
                amat(i,i) = 1d0
            end do
            call dsyrk('l', 'n', k, p, 1d0, yb8, k, dble(inflat), amat, k)
            call dcopy(k*k, amat, 1, evect, 1)
            call dsyevd('v', 'l', k, evect, k, eval, work, lwork, iwork, liwork, info)
            lam = eval
            xa = letkf_solve(xb, yo, yb, inflat, irtpp /= 0, rtpp_a, irtps /= 0, rtps_a)
            write(21) xa, lam
            deallocate(yo, yb, yb8)
        end do
        close(40)
        close(21)
    end subroutine do_solve

    ! get_lz KATs for a single obs type (no Q1 mixing).
    ! in: nobs nq max_lz (i4) hclr vclr (r4) xyz(3,nobs) q(3,nq) (r4)
    ! out: per query nfound (i4) idx(max_lz) (i4, 1-based, 0 padded) r2(max_lz) (r4)
    subroutine do_search
        integer :: nobs, nq, max_lz, dim, iq, nlz
        real    :: hclr, vclr, hclr_inv, vclr_inv
        real, parameter :: r2 = gc1999 * gc1999             ! module_localization.f90:202
        real, allocatable :: xyz(:,:), q(:,:)
        real    :: tmp(3)
        type(kdtree2), pointer :: tree
        type(kdtree2_result), allocatable :: results(:)
        integer, allocatable :: idx(:)
        real,    allocatable :: dis(:)
        open(40, file=trim(fin), access='stream', form='unformatted', status='old')
        read(40) nobs, nq, max_lz
        read(40) hclr, vclr
        allocate(xyz(3,nobs), q(3,nq), results(max_lz), idx(max_lz), dis(max_lz))
        read(40) xyz, q
        close(40)
        ! build_tree normalisation, module_localization.f90:76-82, 148-160
        hclr_inv = 1.0 / (hclr * 1e3)
        if (vclr > 0.) then
            vclr_inv = 1.0 / (vclr * 1e3)
        else
            vclr_inv = -1.
        end if
        xyz(1:2,:) = xyz(1:2,:) * hclr_inv
        if (vclr_inv > 0.) then
            dim = 3
            xyz(3,:) = xyz(3,:) * vclr_inv
        else
            dim = 2
            xyz(3,:) = -1.
        end if
        ! Q7: with dim = 2, kdtree2_create copies the_data(:,ind(i)) (3 rows) into
        ! rearranged_data(2,n) (module_kdtree2.f90:671-675) — flang's runtime rejects that
        ! shape mismatch, so pass the two rows the tree actually reads (same tree, same search).
        if (dim == 3) then
            tree => kdtree2_create(xyz, dim=dim)
        else
            tree => kdtree2_create(xyz(1:2,:), dim=dim)
        end if
        open(21, file=trim(fout), access='stream', form='unformatted', status='replace')
        do iq = 1, nq
            ! get_lz, module_localization.f90:243-253
            tmp(1:2) = q(1:2,iq) * hclr_inv
            if (vclr_inv > 0.) then
                tmp(3) = q(3,iq) * vclr_inv
                call kdtree2_r_nearest(tree, tmp(1:3), r2, nlz, max_lz, results)
            else
                call kdtree2_r_nearest(tree, tmp(1:2), r2, nlz, max_lz, results)
            end if
            idx = 0
            dis = 0.
            if (nlz > 0) then
                idx(1:nlz) = results(1:nlz) % idx
                dis(1:nlz) = results(1:nlz) % dis
            end if
            write(21) nlz, idx, dis
        end do
        close(21)
        call kdtree2_destroy(tree)
    end subroutine do_search

    subroutine do_gc
        integer :: n, i
        real, allocatable :: x(:), y(:)
        open(40, file=trim(fin), access='stream', form='unformatted', status='old')
        read(40) n
        allocate(x(n), y(n))
        read(40) x
        close(40)
        do i = 1, n
            y(i) = Gaspari_Cohn_1999(x(i))
        end do
        open(21, file=trim(fout), access='stream', form='unformatted', status='replace')
        write(21) y
        close(21)
    end subroutine do_gc

    ! letkf_tune_q KATs.  in: k nx ny nz (i4), q(nx,ny,nz,k) (r4).  out: q after the call
    subroutine do_tuneq
        integer :: k, nx, ny, nz
        real, allocatable :: q(:,:,:,:)
        open(40, file=trim(fin), access='stream', form='unformatted', status='old')
        read(40) k, nx, ny, nz
        call setup_k(k)
        allocate(q(nx, ny, nz, k))
        read(40) q
        close(40)
        call letkf_tune_q(nz, q)
        open(21, file=trim(fout), access='stream', form='unformatted', status='replace')
        write(21) q
        close(21)
    end subroutine do_tuneq

    include 'ref_driver.inc'

end module harness_lib

program ref_harness
    use harness_lib
    implicit none
    character(len=512) :: mode

    call get_command_argument(1, mode)
    call get_command_argument(2, fin)
    call get_command_argument(3, fout)

    select case (trim(mode))
    case ('consts')
        call do_consts
    case ('solve')
        call do_solve
    case ('search')
        call do_search
    case ('gc')
        call do_gc
    case ('driver')
        call do_driver
    case ('tuneq')
        call do_tuneq
    case default
        stop "ref_harness: unknown mode"
    end select
end program ref_harness
